#!/bin/bash
# GPU tests + smoke, then bench.py lines of the small shapes with the automatic
# product-stream priority (gemm_priority -1) against priority forced off (0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
  tail -1 gpurun_out/smoke.log
fi
: > gpurun_out/gp_bench.jsonl
for rep in 1 2; do
for a in "--n 512 --p 32" "--n 512 --p 32 --opt gemm_priority=0" "--n 768 --p 63" "--n 768 --p 63 --opt gemm_priority=0"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/gp_one.json 2>> gpurun_out/gp_bench.err || exit 3
  cat gpurun_out/gp_one.json >> gpurun_out/gp_bench.jsonl
  echo "$a $(python3 -c "import json,sys; d=json.load(open('gpurun_out/gp_one.json')); print(d['ms_per_step'], round(d['value']/1e9,1))")"
done
done
