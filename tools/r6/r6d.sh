#!/bin/bash
# Round-6 fourth GPU call: parity of the new options, then interleaved A/B of
# row-scan wave priority (scan_prio) and XCD-contiguous stage blocks
# (stage_xcd) with 256 / 128 / 64-element stage blocks, at 1024^2 P=63,
# 512^2 P=32 and on the 8-way shard rank.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options or gemm_kern" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
V="--variant base: --variant sp3:scan_prio=3 --variant x:stage_xcd=1 --variant e128x:stage_elems=128,stage_xcd=1 --variant e128xp:stage_elems=128,stage_xcd=1,scan_prio=3 --variant e64x:stage_elems=64,stage_xcd=1 --variant e64xp:stage_elems=64,stage_xcd=1,scan_prio=3"
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 5 --steps 10 $V > $O/ab1024.txt 2> $O/ab1024.err
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 5 --steps 20 $V > $O/ab512.txt 2> $O/ab512.err
for r in 1 2; do for o in "scan_prio=0" "scan_prio=3" "stage_xcd=1" "stage_xcd=1 --opt stage_elems=64 --opt scan_prio=3"; do
  n=$(echo $o | tr -c 'a-z0-9' '_')
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 --opt $o > $O/s8_${n}_$r.json 2>> $O/s8.err
done; done
echo r6d done
