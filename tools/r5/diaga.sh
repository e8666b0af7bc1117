#!/bin/bash
# round 5: the stage kernel's phase-A share (timing diagnostic: cells wrong)
set -o pipefail
out=gpurun_out/${1:-r5af}
mkdir -p $out
V="--variant base: --variant noA:stage_diag_a=1 --variant noload:stage_diag_a=2"
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 --variant sbase:overlap=0,phase1_overlap=0,pipeline=0 --variant snoA:overlap=0,phase1_overlap=0,pipeline=0,stage_diag_a=1 --variant snoload:overlap=0,phase1_overlap=0,pipeline=0,stage_diag_a=2 > $out/ab1024_serial.txt 2>&1 || exit $?
echo diaga done
