#!/bin/bash
# GPU tests, then rank 0 of an 8-way row shard (1024^2 P=63) under option variants.
# Usage: bash tools/probe_shard.sh "opt=v opt=v" "opt=v" ...   ("" = defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
i=0
for v in "$@"; do
  i=$((i+1)); args=""
  for kv in $v; do args="$args --opt $kv"; done
  timeout -k 10 200 python tools/shard_sim.py --worlds ${WORLDS:-8} --rank 0 --steps 10 $args > gpurun_out/ps_$i.json 2>&1 || exit $?
  echo "rep $rep [$v] $(grep -h step_ms gpurun_out/ps_$i.json | tr -d ' \n')"
done
done
