#!/bin/bash
# Round-6: place_trials (best of k placements of each >= 1 GiB cell stream) in fresh bench processes
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6pt}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "place_trials or tuning_options" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
A="--no-check --no-ingest --no-cpu-baseline --no-profile"
for r in 1 2 3; do for k in 0 3; do
  SVDW_HOST_TRACE=0 timeout -k 10 200 python3 bench.py $A --opt place_trials=$k > $O/b_k${k}_$r.json 2>> $O/e.err
done; done
SVDW_HOST_TRACE=1 timeout -k 10 200 python3 bench.py $A --steps 5 --opt place_trials=4 > $O/b_trace.json 2> $O/trace.err
for r in 1 2; do for k in 0 3; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 $A --opt place_trials=$k > $O/b512_k${k}_$r.json 2>> $O/e.err
done; done
echo r6pt done
