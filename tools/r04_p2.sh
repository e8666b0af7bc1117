#!/bin/bash
# Round-4 probe: config-2 host time and two-context alternation; steady-state
# (no hold) kernel traces of pipelined witnesses at 1024^2, 512^2, 8-way rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_parity_gpu.py tests/test_verify_mul_config.py tests/test_graph_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 9; }
tail -1 $O/pytest.log
for i in 1 2; do
  for l in 1 2; do
    timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline --opt lanes=$l > $O/vm_l${l}_$i.json 2>> $O/vm.err || exit 8
  done
done
timeout -k 10 200 python tools/probes/vmhost.py > $O/vmhost.json 2> $O/vmhost.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ss_1024 -o run -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest > /dev/null 2> $O/ss_1024.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ss_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 8 > /dev/null 2> $O/ss_s8.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ss_512 -o run -- python3 bench.py --n 512 --p 32 --steps 8 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest > /dev/null 2> $O/ss_512.err || exit 4
echo done
