#!/bin/bash
# Round-6: stage_rot (phase B from a block-dependent window) across placements
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6rot}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options or full_size_sampled or pipelined" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 500 python3 tools/r6/place_ab.py > $O/pa1024.jsonl 2> $O/e.err
PA_N=512 PA_P=32 PA_STEPS=60 timeout -k 10 300 python3 tools/r6/place_ab.py > $O/pa512.jsonl 2>> $O/e.err
echo r6rot done
