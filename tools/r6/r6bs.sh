#!/bin/bash
# Round-6: bench.py against shard_sim.py's one-rank witness on one box, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6bs}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-check --no-ingest --no-cpu-baseline --no-profile > $O/bench_$r.json 2>> $O/e.err
  timeout -k 10 200 python3 tools/shard_sim.py --worlds 1 --steps 30 > $O/sim_$r.json 2>> $O/e.err
  timeout -k 10 200 python3 tools/r6/order.py --first tensors > $O/order_$r.json 2>> $O/e.err
done
timeout -k 10 200 python3 bench.py > $O/bench_full.json 2>> $O/e.err
echo r6bs done
