#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6r3}
mkdir -p $O
(timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1) || true
REALLOC_N=7 timeout -k 10 400 python3 tools/r6/realloc.py > $O/realloc.jsonl 2> $O/e.err
echo r6r3 done
