#!/bin/bash
# round 5: dependency events of the product chain recorded by the kernels'
# dispatch (bind_deps) -- parity, then the 8-way rank, 512^2 and 1024^2
set -o pipefail
out=gpurun_out/${1:-r5ag}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pipelined or tuning or shard_rank" > $out/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  for x in 0 1; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 40 --opt bind_deps=$x > $out/s8_b${x}_$r.json 2>> $out/s8.err || exit $?
  done
done
V="--variant base: --variant bd:bind_deps=1"
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 7 --steps 20 $V > $out/ab512.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 6 $V > $out/ab1024.txt 2>&1 || exit $?
echo bind done
