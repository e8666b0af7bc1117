#!/bin/bash
# Round-6: wide-tile CRT GEMM parity (engine) and probe
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6y}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu -k "persistent or gemm_kern or tuning_options or full_size_shard or crt_gemm or honest" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
echo r6y done
