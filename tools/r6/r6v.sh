#!/bin/bash
# Round-6: RCCL group before / after the engine context, and none (tools/r6/rccl1.py)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6v}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for v in "0 0" "1 0" "1 1"; do set -- $v
  timeout -k 10 200 python3 tools/r6/rccl1.py --dist $1 --ctx-first $2 >> $O/rccl1024.jsonl 2>> $O/e.err
  timeout -k 10 200 python3 tools/r6/rccl1.py --dist $1 --ctx-first $2 --shard 8 --steps 60 >> $O/rccl_s8.jsonl 2>> $O/e.err
done; done
echo r6v done
