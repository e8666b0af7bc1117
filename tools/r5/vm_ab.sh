#!/bin/bash
# config 2 (verify_mul 256^2 P=32): captured graph on one stream (vm_linear 1) vs forked (0), alternating runs
set -o pipefail
out=gpurun_out/${1:-vm}
mkdir -p $out
: > $out/vm.jsonl
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --workload verify_mul --steps 200 --warmup 20 --no-cpu-baseline --no-check --no-ingest --opt vm_linear=$v > $out/vm_$v.json 2>> $out/vm.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$out/vm_$v.json')); print(json.dumps({'vm_linear': $v, 'ms': d['ms_per_step'], 'host': d.get('host_enqueue_ms_per_step')}))" >> $out/vm.jsonl
  done
done
