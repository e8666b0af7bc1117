#!/bin/bash
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6pp}
mkdir -p $O
REALLOC_N=7 timeout -k 10 400 python3 tools/r6/placeprobe.py > $O/pp.jsonl 2> $O/e.err
echo r6pp done
