#!/bin/bash
# Round-6: an RCCL process group (world 1) initialised before the context vs none
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6u}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for dd in 0 1; do
  timeout -k 10 200 python3 tools/r6/rccl1.py --dist $dd >> $O/rccl1024.jsonl 2>> $O/e.err
  timeout -k 10 200 python3 tools/r6/rccl1.py --dist $dd --shard 8 --steps 60 >> $O/rccl_s8.jsonl 2>> $O/e.err
done; done
echo r6u done
