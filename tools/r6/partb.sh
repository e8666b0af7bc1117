#!/bin/bash
# final_r06.sh part b, then the row-scan probe (tools/probes/scanprobe).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PART=b bash tools/final_r06.sh || exit $?
mkdir -p gpurun_out/r6i
timeout -k 10 120 tools/probes/scanprobe 3 10 > gpurun_out/r6i/scan3.txt 2>&1 || exit 20
timeout -k 10 120 tools/probes/scanprobe 6 10 > gpurun_out/r6i/scan6.txt 2>&1 || exit 21
echo partb+scan done
