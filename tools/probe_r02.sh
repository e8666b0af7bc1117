#!/bin/bash
# Round-2 probe: shard simulation, sharded-rank timeline, small-witness timeline,
# verify_mul (config 2) bench line. Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/shard_sim.py --worlds 1,2,4,8 --steps 5 > gpurun_out/shard_sim.json 2>gpurun_out/shard_sim.err || exit $?
cat gpurun_out/shard_sim.json | tr -d '\n' | head -c 1500; echo
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_shard8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 > /dev/null 2>gpurun_out/prof_shard8.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_512 -o run -- python3 bench.py --n 512 --p 32 --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check > gpurun_out/prof_512.json 2>gpurun_out/prof_512.err || exit $?
timeout -k 10 300 python bench.py --n 512 --p 32 --steps 20 --warmup 5 --no-cpu-baseline --no-check > gpurun_out/bench_512.json 2>gpurun_out/bench_512.err || exit $?
timeout -k 10 300 python bench.py --workload verify_mul --steps 20 --warmup 5 > gpurun_out/bench_vm.json 2>gpurun_out/bench_vm.err || exit $?
cat gpurun_out/bench_512.json gpurun_out/bench_vm.json
