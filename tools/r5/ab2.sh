#!/bin/bash
# round 5: stage-kernel variants at 1024^2 / 512^2 (tools/ab.py, one process each)
# and the 8-way rank with small launches spread or not (tools/shard_sim.py)
set -o pipefail
out=gpurun_out/${1:-r5g}
mkdir -p $out
V=${V:-"--variant old:stage_occ=0"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
if [ -n "${S8:-}" ]; then
  for r in 1 2; do
    for sp in 1 0; do
      timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 20 --opt stage_occ=0 --opt small_spread=$sp > $out/s8_sp${sp}_$r.json 2>> $out/s8.err || exit $?
    done
  done
fi
