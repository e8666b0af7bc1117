#!/bin/bash
# Round-6: the 256 x 128 tile CRT GEMM (k_gemm_crt_wide) in the probe, 1024 and
# odd tile-row counts (640: 5 tile rows; 900: 8)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6x}
mkdir -p $O
timeout -k 10 150 tools/probes/gemmprobe 640 10 > $O/gemm640.txt 2>&1
timeout -k 10 150 tools/probes/gemmprobe 1024 20 > $O/gemm1024.txt 2>&1
timeout -k 10 150 tools/probes/gemmprobe 2048 10 > $O/gemm2048.txt 2>&1
echo r6x done
