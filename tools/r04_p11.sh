#!/bin/bash
# Round-4 probe: config 2 with a linear launch graph (side streams off) vs the
# forked one, with two lanes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p11
mkdir -p $O
export TMPDIR=/tmp
: > $O/res.txt
for round in 1 2; do
  for v in "" "--opt phase1_overlap=0" "--opt overlap=0" "--opt phase1_overlap=0 --opt overlap=0"; do
    r=$(timeout -k 10 200 python bench.py --workload verify_mul --no-cpu-baseline --no-check --steps 200 $v 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])") || exit 1
    echo "round $round [$v] $r" >> $O/res.txt
  done
done
echo done
