#!/bin/bash
# Round-6 first GPU call: CRT GEMM probe (alone and beside a stand-in store
# stream), store-pattern probe 11, then the round-4 / round-5 same-box A/B.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6a}
mkdir -p $O
timeout -k 10 150 tools/probes/gemmprobe 1024 20 > $O/gemm.txt 2>&1
timeout -k 10 300 tools/probes/storepat11 > $O/sp11.txt 2>&1
timeout -k 10 700 bash tools/r6/ab45.sh $O/ab45 3
