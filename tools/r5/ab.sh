#!/bin/bash
# round 5: same-process A/B of the stage kernels (tools/ab.py), then the GPU suite
set -o pipefail
out=gpurun_out/${1:-r5b}
shift
mkdir -p $out
V=${V:-"--variant old:stage_occ=0 --variant p1:stage_occ=1 --variant p2:stage_occ=2 --variant p3:stage_occ=3"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
if [ -n "${SUITE:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $out/pytest.log; exit $rc
fi
