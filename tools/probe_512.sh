#!/bin/bash
# bench.py lines at 512^2 P=32 (BASELINE config 3) under scheduling options.
# Usage: bash tools/probe_512.sh "" "res_first=1" "p1_at=0 gemm_batch=0" ...  ("" = defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for o in "$@"; do
  args=""; for kv in $o; do args="$args --opt $kv"; done
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --n 512 --p 32 --steps 20 $args > gpurun_out/p512.json 2>> gpurun_out/p512.err || exit 3
  echo "[$o] $(python3 -c "import json,sys; d=json.load(open('gpurun_out/p512.json')); print(d['ms_per_step'], round(d['value']/1e9,1))")"
done
done
