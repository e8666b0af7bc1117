#!/bin/bash
# round 5: steady-state kernel traces of pipelined 1024^2 witnesses, plain vs non-temporal stage stores
set -o pipefail
out=gpurun_out/${1:-r5k}
mkdir -p $out
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-profile --no-check --no-ingest"
for v in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/nt$v -o run -- python3 bench.py --steps 12 --warmup 3 $NB --opt stage_nt=$v > $out/nt$v.json 2> $out/nt$v.err || exit $?
done
