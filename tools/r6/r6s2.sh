#!/bin/bash
# Round-6: context-first vs tensors-first process order (tools/r6/order.py),
# alternating, 1024^2 P=63 and 512^2 P=32; bench.py and shard_sim world 1 beside.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6s2}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for f in ctx tensors setdev; do
  timeout -k 10 200 python3 tools/r6/order.py --first $f >> $O/order1024.jsonl 2>> $O/e.err
  timeout -k 10 200 python3 tools/r6/order.py --first $f --n 512 --p 32 --steps 60 >> $O/order512.jsonl 2>> $O/e.err
done; done
timeout -k 10 200 python3 bench.py --no-check --no-ingest --no-cpu-baseline --no-profile > $O/bench1024.json 2>> $O/e.err
timeout -k 10 200 python3 tools/shard_sim.py --worlds 1 --steps 30 > $O/sim1.json 2>> $O/e.err
echo r6s2 done
