#!/bin/bash
# round 5: the stage stream kept off k CUs per 32 (SVDW_CUMASK), with 256- and
# XCD-contiguous 64-element stage blocks; bench.py processes, alternating
set -o pipefail
out=gpurun_out/${1:-r5y}
mkdir -p $out
B="--steps 20 --warmup 4 --no-cpu-baseline --no-ingest --no-profile --no-check"
X64="--opt stage_elems=64 --opt stage_xcd=1"
for r in 1 2; do
  for cfg in "base:0:" "x64:0:$X64" "cm4:4:" "x64cm4:4:$X64" "x64cm8:8:$X64" "x64cm2:2:$X64"; do
    name=${cfg%%:*}; rest=${cfg#*:}; k=${rest%%:*}; opts=${rest#*:}
    SVDW_CUMASK=$k timeout -k 10 120 python3 bench.py $B $opts > $out/n1024_${name}_$r.json 2> $out/n1024_${name}_$r.err || exit $?
    SVDW_CUMASK=$k timeout -k 10 120 python3 bench.py --n 512 --p 32 $B $opts > $out/n512_${name}_$r.json 2> $out/n512_${name}_$r.err || exit $?
  done
done
echo cumask done
