#!/bin/bash
# Parity subset, then bench.py lines with the CRT combine via LDS for symmetric
# batches (comb_direct 1, default) against direct stores everywhere (2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sharded or cell_stream or tuning" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for rep in 1 2; do
for s in "--n 512 --p 32" "--n 1024 --p 63"; do
for o in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-check $s --steps 20 --opt comb_direct=$o > gpurun_out/pc.json 2>> gpurun_out/pc.err || exit 3
  echo "[$s comb_direct=$o] $(python3 -c "import json,sys; d=json.load(open('gpurun_out/pc.json')); print(d['ms_per_step'], round(d['value']/1e9,1))")"
done
done
done
