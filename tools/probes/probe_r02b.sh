#!/bin/bash
# Priority / placement options on the latency-bound shapes: rank 0 of an 8-way
# 1024^2 P=63 row shard (tools/probes/probe_shard.sh) and 512^2 P=32 (tools/ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
SKIP_TESTS=1 bash tools/probes/probe_shard.sh "" "stage_priority=1" "gemm_priority=1" "stage_priority=1 gemm_priority=1" "p1_at=3" || exit $?
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 --variant base: \
  --variant sp:stage_priority=1 --variant gp:gemm_priority=1 --variant pa0:prelaunch_at=1 > gpurun_out/ab512.txt 2>&1 || exit $?
cat gpurun_out/ab512.txt | head -20
