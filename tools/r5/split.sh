#!/bin/bash
# round 5: split-K of small CRT products -- parity (whole GPU suite), then A/B
# on the 8-way rank (tools/shard_sim.py) and at 512^2 / 1024^2 (tools/ab.py)
set -o pipefail
out=gpurun_out/${1:-r5l}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for sp in 1 0; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 20 --opt gemm_split=$sp > $out/s8_sp${sp}_$r.json 2>> $out/s8.err || exit $?
  done
done
V="--variant split:gemm_split=1 --variant nosplit:gemm_split=0" ./tools/r5/ab2.sh ${1:-r5l}
