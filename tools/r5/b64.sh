#!/bin/bash
# round 5: phase-B source words by ds_read_b64 (stage_b64) against the five
# 4-byte reads -- parity of the option, then tools/ab.py at 1024^2 / 512^2 and
# the 8-way rank (tools/shard_sim.py), same process per size
set -o pipefail
out=gpurun_out/${1:-r5m}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "tuning_options or front_streamer" > $out/pytest.log 2>&1 || exit $?
V="--variant old:stage_b64=0 --variant b64:stage_b64=1"
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
for r in 1 2; do
  for b in 0 1; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 20 --opt stage_b64=$b > $out/s8_b${b}_$r.json 2>> $out/s8.err || exit $?
  done
done
echo b64 done
