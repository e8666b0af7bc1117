#!/bin/bash
# Iteration loop on one box: GPU parity tests (pytest -k expr), the shard
# simulation, the 1-GPU bench lines (1024^2 P=63, 512^2 P=32, verify_mul 256^2)
# and the GPU-only schedules of rank 0 of the 8-way shard and of the 1-GPU step.
#   bash tools/r03_iter.sh tag "pytest -k expr" [extra svdw options as k=v ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
K=$2
shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
OPTS=""
for kv in "$@"; do OPTS="$OPTS --opt $kv"; done
if [ -n "$K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 240 python3 tools/shard_sim.py --worlds 1,2,4,8 --steps 10 $OPTS > $O/shard_sim.json 2> $O/shard_sim.err || exit $?
python3 -c "import json; d=json.load(open('$O/shard_sim.json')); [print('shard', k, v['step_ms'], v['rank_ms'], v.get('efficiency_vs_1')) for k,v in d['worlds'].items()]"
for cfg in "--n 1024 --p 63" "--n 512 --p 32" "--workload verify_mul"; do
  timeout -k 10 240 python3 bench.py $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-ingest $OPTS > $O/bench.json 2> $O/bench.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d.get('roofline',{}); print('bench', '$cfg', d['ms_per_step'], round(d['value']/1e9,2), 'G', 'kernel', r.get('kernel'), r.get('frac'), 'step', (r.get('step') or {}).get('frac'), 'check', (d.get('witness_check') or {}).get('ok'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/go_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 $OPTS > /dev/null 2> $O/go_s8.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/go_1k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest --opt hold_us=3000 $OPTS > /dev/null 2> $O/go_1k.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/go_vm -o run -- python3 bench.py --workload verify_mul --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest --opt hold_us=1000 $OPTS > /dev/null 2> $O/go_vm.err || exit $?
for d in go_s8 go_1k go_vm; do
  f=$(ls $O/$d/*/run_kernel_trace.csv 2>/dev/null | head -n 1)
  [ -z "$f" ] && f=$(ls $O/$d/run_kernel_trace.csv)
  python3 tools/timeline.py "$f" --all > $O/$d.timeline.txt || exit $?
  head -16 $O/$d.timeline.txt
done
