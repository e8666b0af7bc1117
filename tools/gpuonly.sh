#!/bin/bash
# GPU-only schedules (hold_us: the host has enqueued the whole step before it
# runs) of 512^2 P=32, rank 0 of an 8-way 1024^2 P=63 shard and 1024^2 P=63.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
H=${HOLD:-1500}
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/go_512 -o run -- python3 bench.py --n 512 --p 32 --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --opt hold_us=$H > /dev/null 2>gpurun_out/go_512.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/go_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=$H > /dev/null 2>gpurun_out/go_s8.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/go_1024 -o run -- python3 bench.py --n 1024 --p 63 --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --opt hold_us=$H > /dev/null 2>gpurun_out/go_1024.err || exit $?
