#!/bin/bash
# Round-6 A/B: stage blocks running several chunks (stage_chunks 2 / 4, the
# next chunk's view loads ahead of the current chunk's stores) against one
# chunk per block; plus bench lines at 10 and 50 steps (pipeline fill/drain).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6l}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options or stage_chunks or pipelined" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
V="--variant c1:stage_chunks=1 --variant c2:stage_chunks=2 --variant c4:stage_chunks=4"
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 6 --steps 10 $V > $O/ab1024.txt 2> $O/ab1024.err
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 6 --steps 20 $V > $O/ab512.txt 2> $O/ab512.err
for r in 1 2; do for o in 1 2 4; do
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 --opt stage_chunks=$o > $O/s8_c${o}_$r.json 2>> $O/s8.err
done; done
for r in 1 2; do for s in 10 50; do
  timeout -k 10 200 python3 bench.py --steps $s --no-check --no-ingest --no-cpu-baseline --no-profile > $O/b1024_s${s}_$r.json 2>> $O/b.err
done; done
echo r6l done
