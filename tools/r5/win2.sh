#!/bin/bash
# round 5: k_stage_win with more windows per block (tools/ab.py, 1024^2 / 512^2)
set -o pipefail
out=gpurun_out/${1:-r5o}
mkdir -p $out
V=${V:-"--variant old:stage_win=0 --variant w32s8:stage_win=32,stage_win_sb=8 --variant w32s256:stage_win=32,stage_win_sb=256 --variant w64s8:stage_win=64,stage_win_sb=8 --variant w64s64:stage_win=64,stage_win_sb=64"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
echo win2 done
