#!/bin/bash
# round 5: window-interleaved stage kernel (stage_win) -- parity, then
# tools/ab.py at 1024^2 / 512^2 against the one-chunk-per-block kernels
set -o pipefail
out=gpurun_out/${1:-r5n}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "window_stage or tuning_options or pipelined_full_size" > $out/pytest.log 2>&1 || exit $?
V=${V:-"--variant old:stage_win=0 --variant w8:stage_win=8,stage_win_sb=8 --variant w8s128:stage_win=8,stage_win_sb=128 --variant w16s256:stage_win=16,stage_win_sb=256"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
echo win done
