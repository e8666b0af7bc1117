#!/bin/bash
# Round-6: bench.py against tools/ab.py on one box at 512^2 P=32 (VERDICT #4:
# is the bench line's gap to the A/B medians real?), bench.py at 10 / 30
# steps at 1024^2, and an 8-round 1024^2 A/B with samples in run order
# (does the step drift as the box warms?).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6m}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile > $O/b512_$r.json 2>> $O/b.err
  timeout -k 10 200 python3 tools/ab.py --n 512 --p 32 --rounds 3 --steps 40 > $O/ab512_$r.txt 2>> $O/ab.err
done
for r in 1 2; do for s in 10 30; do
  timeout -k 10 200 python3 bench.py --steps $s --no-check --no-ingest --no-cpu-baseline --no-profile > $O/b1024_s${s}_$r.json 2>> $O/b.err
done; done
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 12 --steps 10 > $O/ab1024_drift.txt 2>> $O/ab.err
echo r6m done
