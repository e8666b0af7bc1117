#!/bin/bash
# Round-6: place_trials default 3 vs 0: fresh bench processes, the 8-way rank, 2048x1024
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6pt2}
mkdir -p $O
A="--no-check --no-ingest --no-cpu-baseline --no-profile"
for r in 1 2; do for k in 3 0; do
  timeout -k 10 200 python3 bench.py $A --opt place_trials=$k > $O/b_k${k}_$r.json 2>> $O/e.err
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 60 --opt place_trials=$k > $O/s8_k${k}_$r.json 2>> $O/e.err
  timeout -k 10 200 python3 bench.py --n 2048 --m 1024 --p 32 $A --opt place_trials=$k > $O/b2048_k${k}_$r.json 2>> $O/e.err
done; done
echo r6pt2 done
