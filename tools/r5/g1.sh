#!/bin/bash
# round 5: k_gamma_prep on st3 (gamma_at 1) at 1024^2 / 512^2 and the 8-way
# rank with worlds 1 and 8 (efficiency on one box)
set -o pipefail
out=gpurun_out/${1:-r5q}
mkdir -p $out
V="--variant base: --variant g1:gamma_at=1 --variant d1g1:dchk_at=1,gamma_at=1"
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
for r in 1 2; do
  for g in 0 1; do
    timeout -k 10 300 python tools/shard_sim.py --worlds 1,8 --steps 20 --opt gamma_at=$g > $out/sw_g${g}_$r.json 2>> $out/sw.err || exit $?
  done
done
echo g1 done
