#!/bin/bash
# round 5: front streamer parity, then A/B against the block kernel
set -o pipefail
out=gpurun_out/${1:-r5h}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread -k "front_streamer or tuning_options or pipelined_full_size" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/pytest.log; [ $rc -eq 0 ] || exit $rc
V=${V:-"--variant old:stage_occ=0 --variant f1:stage_occ=1"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1
