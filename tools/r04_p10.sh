#!/bin/bash
# Round-4 probe: a high-priority cell stream (created with the context) for the
# pipelined witness, whose cell stream carries the next call's product chain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p10
mkdir -p $O
export TMPDIR=/tmp
: > $O/res.txt
for round in 1 2; do
  for pr in 0 1; do
    for a in "--n 512 --p 32" "--n 1024 --p 63"; do
      r=$(SVDW_CELL_PRIORITY=$pr timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-check --no-ingest --no-profile --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
      echo "round $round prio $pr [$a] $r" >> $O/res.txt
    done
    for rk in 0 5; do
      ms=$(SVDW_CELL_PRIORITY=$pr timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $rk --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 2
      echo "round $round prio $pr [s8 rank $rk] $ms" >> $O/res.txt
    done
  done
done
echo done
