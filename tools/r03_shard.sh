#!/bin/bash
# Row-sharded iteration loop: sharded parity tests, the shard simulation and
# the GPU-only schedule of rank 0 of the 8-way shard (hold_us).
#   bash tools/r03_shard.sh [tag] [pytest -k expr] [extra shard_sim args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-s}
K=${2:-"sharded or products_on_cell"}
shift $(( $# < 2 ? $# : 2 ))
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python3 tools/shard_sim.py --worlds 1,2,4,8 --steps 10 "$@" > $O/shard_sim.json 2> $O/shard_sim.err || exit $?
python3 -c "import json; d=json.load(open('$O/shard_sim.json')); [print(k, v['step_ms'], v['rank_ms'], v.get('efficiency_vs_1')) for k,v in d['worlds'].items()]"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/go_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 "$@" > /dev/null 2> $O/go_s8.err || exit $?
f=$(ls $O/go_s8/*/run_kernel_trace.csv 2>/dev/null | head -n 1)
[ -z "$f" ] && f=$(ls $O/go_s8/run_kernel_trace.csv)
python3 tools/timeline.py "$f" --all > $O/go_s8.timeline.txt && cat $O/go_s8.timeline.txt
