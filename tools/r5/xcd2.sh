#!/bin/bash
# round 5: XCD-contiguous 64-element chunks with the stage blocks per CU capped
# through an LDS floor (stage_lds_floor)
set -o pipefail
out=gpurun_out/${1:-r5u}
mkdir -p $out
V=${V:-"--variant base: --variant x64:stage_xcd=1,stage_elems=64 --variant x64f4:stage_xcd=1,stage_elems=64,stage_lds_floor=40960 --variant x64f3:stage_xcd=1,stage_elems=64,stage_lds_floor=53248 --variant x64f2:stage_xcd=1,stage_elems=64,stage_lds_floor=81920 --variant e64:stage_elems=64"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
echo xcd2 done
