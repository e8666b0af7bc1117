#!/bin/bash
# round 5: smaller stage blocks capped by an LDS floor that leaves one row-scan
# block (27 KB LDS) room on every CU
set -o pipefail
out=gpurun_out/${1:-r5ac}
mkdir -p $out
V="--variant base: --variant e128f42:stage_elems=128,stage_lds_floor=43008 --variant e64f42:stage_elems=64,stage_lds_floor=43008 --variant e128f54:stage_elems=128,stage_lds_floor=55296 --variant e192:stage_elems=192"
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 20 $V > $out/ab512.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 || exit $?
echo occ done
