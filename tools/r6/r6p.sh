#!/bin/bash
# Round-6: bench.py 512^2 P=32 with 3 / 4 / 10 warm-up steps, alternating
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6p}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for w in 3 4 10; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 --warmup $w --no-check --no-ingest --no-cpu-baseline --no-profile > $O/b512_w${w}_$r.json 2>> $O/b.err
done; done
echo r6p done
