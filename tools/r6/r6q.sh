#!/bin/bash
# Round-6: bench.py 512^2 P=32 and 1024^2 with and without the hold checkpoints
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6q}
mkdir -p $O
export TMPDIR=/tmp
A="--steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile"
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 $A > $O/b512_hold_$r.json 2>> $O/b.err
  timeout -k 10 200 python3 tools/r6/nohold.py --n 512 --p 32 $A > $O/b512_nohold_$r.json 2>> $O/b.err
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/b1024_hold_$r.json 2>> $O/b.err
  timeout -k 10 200 python3 tools/r6/nohold.py $A > $O/b1024_nohold_$r.json 2>> $O/b.err
done
echo r6q done
