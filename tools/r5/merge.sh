#!/bin/bash
# round 5: bounds, diff and ids of a pipelined witness in one st2 launch
# (st2_merge) -- parity, then tools/ab.py at 512^2 / 1024^2 and the 8-way rank
set -o pipefail
out=gpurun_out/${1:-r5x}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pipelined" > $out/pytest.log 2>&1 || exit $?
V="--variant base: --variant m2:st2_merge=1"
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 7 --steps 20 $V > $out/ab512.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 2048 --m 1024 --p 32 --rounds 3 --steps 3 $V > $out/ab2048.txt 2>&1 || exit $?
for r in 1 2; do
  for x in 0 1; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 40 --opt st2_merge=$x > $out/s8_m${x}_$r.json 2>> $out/s8.err || exit $?
  done
done
echo merge done
