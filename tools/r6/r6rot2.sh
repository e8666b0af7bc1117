#!/bin/bash
# Round-6: stage_rot, more placements (variant order alternating), 2048x1024, the 8-way rank, bench lines
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6rot2}
mkdir -p $O
PA_ROUNDS=4 VARIANTS="rot0:stage_rot=0;rot1:stage_rot=1;rot1b:stage_rot=1;rot0b:stage_rot=0" timeout -k 10 600 python3 tools/r6/place_ab.py > $O/pa1024.jsonl 2> $O/e.err
PA_N=2048 PA_P=32 PA_STEPS=10 PA_ROUNDS=3 timeout -k 10 500 python3 tools/r6/place_ab.py > $O/pa2048.jsonl 2>> $O/e.err
for r in 1 2; do for o in 0 1; do
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 60 --opt stage_rot=$o > $O/s8_r${o}_$r.json 2>> $O/e.err
done; done
for r in 1 2; do for o in 0 1; do
  timeout -k 10 200 python3 bench.py --no-check --no-ingest --no-cpu-baseline --no-profile --opt stage_rot=$o > $O/b1024_r${o}_$r.json 2>> $O/e.err
done; done
echo r6rot2 done
