#!/bin/bash
# round 5: tail waits of a pipelined witness on the cell stream only (tail_lite)
set -o pipefail
out=gpurun_out/${1:-r5z}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pipelined" > $out/pytest.log 2>&1 || exit $?
V="--variant base: --variant tl:tail_lite=1"
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 9 --steps 20 $V > $out/ab512.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 7 --steps 6 $V > $out/ab1024.txt 2>&1 || exit $?
for r in 1 2; do
  for x in 0 1; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 40 --opt tail_lite=$x > $out/s8_t${x}_$r.json 2>> $out/s8.err || exit $?
  done
done
echo tail done
