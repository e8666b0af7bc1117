#!/bin/bash
# Round-6: GPU_MAX_HW_QUEUES 4 (the box default) vs 8 with and without an RCCL
# group in the process (tools/r6/rccl1.py), 1024^2 and the 8-way rank
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6w}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for q in 4 8; do for v in "0 0" "1 0" "1 1"; do set -- $v
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 tools/r6/rccl1.py --dist $1 --ctx-first $2 > $O/t.json 2>> $O/e.err
  echo "{\"q\": $q, \"r\": $(cat $O/t.json)}" >> $O/rccl1024.jsonl
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 tools/r6/rccl1.py --dist $1 --ctx-first $2 --shard 8 --steps 60 > $O/t.json 2>> $O/e.err
  echo "{\"q\": $q, \"r\": $(cat $O/t.json)}" >> $O/rccl_s8.jsonl
done; done; done
for r in 1 2; do for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile > $O/t.json 2>> $O/e.err
  echo "{\"q\": $q, \"b512\": $(python3 -c "import json;print(json.load(open('$O/t.json'))['ms_per_step'])")}" >> $O/bench.jsonl
done; done
echo r6w done
