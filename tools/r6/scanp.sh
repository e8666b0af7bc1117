#!/bin/bash
# row-scan probe (tools/probes/scanprobe): 3 and 6 jobs of 1024 rows
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6j}
mkdir -p $O
timeout -k 10 120 tools/probes/scanprobe 3 10 > $O/scan3.txt 2>&1
timeout -k 10 120 tools/probes/scanprobe 6 10 > $O/scan6.txt 2>&1
echo scanp done
