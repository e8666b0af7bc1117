#!/bin/bash
# Round-6 A/B: the pipelined witness's diff + ids held back into the next
# witness's first st2 launch (st2_defer) against one st2 launch each, at
# 1024^2 P=63, 512^2 P=32 and on the 8-way shard rank, plus bench lines.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options or pipelined or lifetime or held_inputs" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
V="--variant d0:st2_defer=0 --variant d1:st2_defer=1"
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 8 --steps 20 $V > $O/ab512.txt 2> $O/ab512.err
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 6 --steps 10 $V > $O/ab1024.txt 2> $O/ab1024.err
for r in 1 2; do for o in 0 1; do
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 --opt st2_defer=$o > $O/s8_d${o}_$r.json 2>> $O/s8.err
done; done
for r in 1 2; do for o in 0 1; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile --opt st2_defer=$o > $O/b512_d${o}_$r.json 2>> $O/b.err
done; done
echo r6h done
