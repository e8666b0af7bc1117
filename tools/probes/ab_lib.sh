#!/bin/bash
# Same-box A/B of two library builds: base (libsvdw_base.so, tools/probes/build_base.sh)
# and the working tree's libsvdw.so, alternating short bench runs.
# Usage (on the GPU box): bash tools/probes/ab_lib.sh [rounds] [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=${1:-3}; shift || true
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  for v in base new; do
    if [ $v = base ]; then lib=$PWD/halo2_svd041_amd/libsvdw_base.so; else lib=$PWD/halo2_svd041_amd/libsvdw.so; fi
    SVDW_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_$v.json 2>/dev/null
    rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; exit $rc; fi
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', i:=$i, round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,2), 'Gcells/s')"
  done
done
