#!/bin/bash
# prod_cell A/B on one box: an 8-way shard rank and 1024^2 / 512^2 unsharded,
# option off vs on, alternating; then the GPU-only timeline of the shard rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for pc in 0 1; do
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 10 --opt prod_cell=$pc > gpurun_out/pc_s8.json 2>&1 || exit $?
    echo "shard8 prod_cell=$pc $(grep -h step_ms gpurun_out/pc_s8.json | tr -d ' \n')"
  done
done
for n in 1024 512; do
  p=63; [ $n = 512 ] && p=32
  for i in 1 2; do
    for pc in 0 1; do
      timeout -k 10 300 python bench.py --n $n --p $p --steps 10 --warmup 3 --no-cpu-baseline --no-check --no-profile --no-ingest --opt prod_cell=$pc > gpurun_out/pc_b.json 2>/dev/null || exit $?
      python -c "import json; d=json.load(open('gpurun_out/pc_b.json')); print('$n prod_cell=$pc', round(d['ms_per_step'],4), 'ms')"
    done
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/go_s8d -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 > /dev/null 2>gpurun_out/go_s8d.err
