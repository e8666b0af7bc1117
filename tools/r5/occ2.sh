#!/bin/bash
# round 5: XCD-contiguous 64 / 128-element stage blocks capped so that one
# row-scan block (27 KB LDS, 128 VGPRs) still fits on every CU
set -o pipefail
out=gpurun_out/${1:-r5ad}
mkdir -p $out
V="--variant base: --variant x64:stage_xcd=1,stage_elems=64 --variant x64f33:stage_xcd=1,stage_elems=64,stage_lds_floor=33792 --variant x64f42:stage_xcd=1,stage_elems=64,stage_lds_floor=43008 --variant x128f42:stage_xcd=1,stage_elems=128,stage_lds_floor=43008"
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 20 $V > $out/ab512.txt 2>&1 || exit $?
echo occ2 done
