#!/bin/bash
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-sp12}
mkdir -p $O
timeout -k 10 120 tools/probes/storepat12 122 4096 > $O/sp12.txt 2>&1
timeout -k 10 120 tools/probes/storepat12 122 4096 > $O/sp12b.txt 2>&1
echo sp12 done
