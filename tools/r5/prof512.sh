#!/bin/bash
# round 5: bench.py at 512^2 P=32 with 40 steps: profiler off / on, alternating
set -o pipefail
out=gpurun_out/${1:-r5aa}
mkdir -p $out
B="--n 512 --p 32 --steps 40 --warmup 5 --no-cpu-baseline --no-ingest --no-check"
for r in 1 2 3; do
  for pf in off on; do
    X=""; [ $pf = off ] && X="--no-profile"
    timeout -k 10 120 python3 bench.py $B $X > $out/n512_${pf}_$r.json 2> $out/n512_${pf}_$r.err || exit $?
  done
done
echo prof512 done
