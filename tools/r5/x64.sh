#!/bin/bash
# round 5: XCD-contiguous 64-element stage blocks (stage_xcd + stage_elems 64)
# against the default, more rounds
set -o pipefail
out=gpurun_out/${1:-r5ae}
mkdir -p $out
V="--variant base: --variant x64:stage_xcd=1,stage_elems=64"
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 9 --steps 6 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 9 --steps 20 $V > $out/ab512.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 2048 --m 1024 --p 32 --rounds 5 --steps 4 $V > $out/ab2048.txt 2>&1 || exit $?
for r in 1 2; do
  for x in 0 1; do
    X=""; [ $x = 1 ] && X="--opt stage_xcd=1 --opt stage_elems=64"
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 40 $X > $out/s8_x${x}_$r.json 2>> $out/s8.err || exit $?
  done
done
echo x64 done
