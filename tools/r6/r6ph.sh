#!/bin/bash
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6ph}
mkdir -p $O
timeout -k 10 500 python3 tools/r6/phase.py > $O/phase1024.jsonl 2> $O/e.err
PHASE_N=512 PHASE_P=32 timeout -k 10 300 python3 tools/r6/phase.py > $O/phase512.jsonl 2>> $O/e.err
echo r6ph done
