#!/bin/bash
# Round-6: completion marks (svdw_mark) in place of the checkpoint side stream:
# tests, then bench.py alternating with tools/r6/benchdiff.py at 512^2 P=32
# and bench.py at 1024^2.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6r}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "marks or held_inputs or lifetime or pipelined or tuning_options" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
A="--steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile"
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 $A > $O/b512_$r.json 2>> $O/b.err
  timeout -k 10 200 python3 tools/r6/benchdiff.py --n 512 --p 32 --steps 40 --rounds 2 > $O/diff512_$r.txt 2>> $O/b.err
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/b1024_$r.json 2>> $O/b.err
done
echo r6r done
