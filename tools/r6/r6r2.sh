#!/bin/bash
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6r2}
mkdir -p $O
timeout -k 10 300 python3 tools/r6/realloc.py > $O/realloc1.jsonl 2> $O/e.err
REALLOC_N=10 timeout -k 10 400 python3 tools/r6/realloc.py > $O/realloc2.jsonl 2>> $O/e.err
echo r6r2 done
