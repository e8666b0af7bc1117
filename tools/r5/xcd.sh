#!/bin/bash
# round 5: XCD-contiguous stage chunks (stage_xcd), with smaller chunks
set -o pipefail
out=gpurun_out/${1:-r5t}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "tuning_options" > $out/pytest.log 2>&1 || exit $?
V=${V:-"--variant base: --variant x:stage_xcd=1 --variant x128:stage_xcd=1,stage_elems=128 --variant x64:stage_xcd=1,stage_elems=64 --variant e128:stage_elems=128"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
for r in 1 2; do
  for x in 0 1; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 40 --opt stage_xcd=$x > $out/s8_x${x}_$r.json 2>> $out/s8.err || exit $?
  done
done
echo xcd done
