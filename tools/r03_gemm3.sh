#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-gemm3}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gemm or sharded or tuning or device_inputs" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for args in "--n 1024" "--n 1024 --sym" "--n 1024 --rows 128"; do
  timeout -k 10 120 python3 tools/gemm_bench.py $args >> $O/gemm.jsonl 2>> $O/gemm.err || exit $?
  timeout -k 10 120 python3 tools/gemm_trace.py $args >> $O/trace.jsonl 2>> $O/gemm.err || exit $?
done
cat $O/gemm.jsonl $O/trace.jsonl
