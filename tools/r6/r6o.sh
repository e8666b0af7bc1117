#!/bin/bash
# Round-6: bench.py (512^2 P=32, 40 steps) alternating with tools/r6/benchdiff.py on one box
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6o}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile > $O/b512_$r.json 2>> $O/b.err
  timeout -k 10 200 python3 tools/r6/benchdiff.py --n 512 --p 32 --steps 40 --rounds 3 > $O/diff512_$r.txt 2>> $O/b.err
done
echo r6o done
