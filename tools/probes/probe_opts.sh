#!/bin/bash
# Same-box option sweep: bench.py at one size with each option set (space-
# separated name=value lists, ';' between sets), alternating, ROUNDS rounds.
# Usage: N=512 P=32 SETS="gemm_batch=1;prod_cell=1" bash tools/probes/probe_opts.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
N=${N:-512}; P=${P:-32}; R=${ROUNDS:-2}
IFS=';' read -ra sets <<< "-;${SETS}"
for i in $(seq 1 "$R"); do
  for s in "${sets[@]}"; do
    args=()
    if [ "$s" != "-" ]; then for o in $s; do args+=(--opt "$o"); done; fi
    timeout -k 10 300 python bench.py --n "$N" --p "$P" --steps 10 --warmup 3 --no-cpu-baseline --no-check \
      --no-profile --no-ingest "${args[@]}" > gpurun_out/po.json 2>/dev/null || exit $?
    python -c "import json; d=json.load(open('gpurun_out/po.json')); print('$N', '[$s]', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,2), 'G')"
  done
done
