#!/bin/bash
# Round-6: place_trials 3 vs 6 vs 0 in fresh bench processes (1024^2)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6pt3}
mkdir -p $O
A="--no-check --no-ingest --no-cpu-baseline --no-profile"
for r in 1 2 3; do for k in 0 3 6; do
  SVDW_HOST_TRACE=1 timeout -k 10 200 python3 bench.py $A --opt place_trials=$k > $O/b_k${k}_$r.json 2> $O/tr_k${k}_$r.err
done; done
echo r6pt3 done
