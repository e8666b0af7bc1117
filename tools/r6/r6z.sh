#!/bin/bash
# Round-6: the wide-tile GEMM inside the 8-way rank's witness (gemm_kern 2) vs per-unit (0)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6z}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for k in 0 2; do
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 60 --opt gemm_kern=$k > $O/s8_k${k}_$r.json 2>> $O/e.err
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 4 --rank 0 --steps 40 --opt gemm_kern=$k > $O/s4_k${k}_$r.json 2>> $O/e.err
done; done
timeout -k 10 150 tools/probes/gemmprobe 1024 20 > $O/gemm1024.txt 2>&1
echo r6z done
