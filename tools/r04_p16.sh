#!/bin/bash
# Round-4 probe: config 2 in bench.py (lanes 1 / 2, 300 steps) beside
# tools/probes/vmstream.py in the same call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p16
mkdir -p $O
export TMPDIR=/tmp
: > $O/res.txt
for round in 1 2; do
  for l in 2 1; do
    r=$(timeout -k 10 200 python bench.py --workload verify_mul --no-cpu-baseline --no-check --steps 300 --opt lanes=$l 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['host_enqueue_ms_per_step'], d['roofline'].get('timing_note','')[-40:])") || exit 1
    echo "round $round lanes $l: $r" >> $O/res.txt
  done
done
timeout -k 10 300 python tools/probes/vmstream.py > $O/vmstream.json 2>> $O/err.txt || exit 2
echo done
