#!/bin/bash
# Captured verify_mul_witness: parity tests, the config-2 bench line with and
# without the graph, host enqueue time, and the graph/event probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/graph
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_verify_mul_config.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline > $O/vm_graph_$i.json 2>> $O/bench.err || exit 3
  timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline --opt graph=0 > $O/vm_eager_$i.json 2>> $O/bench.err || exit 3
done
for f in $O/vm_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['value']/1e9, d['roofline'].get('avg_launch_ms'), d['roofline'].get('timing_note','')[:60])"; done
timeout -k 10 120 python tools/hosttime_vm.py > $O/hosttime.txt 2>&1 || exit 4
cat $O/hosttime.txt
hipcc --offload-arch=gfx950 -O2 tools/graphtest.hip -o $O/graphtest && timeout -k 10 60 $O/graphtest > $O/graphtest.txt 2>&1 || exit 5
cat $O/graphtest.txt
