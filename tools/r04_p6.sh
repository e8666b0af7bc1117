#!/bin/bash
# Round-4 probe: config 2 eager vs graph, one context vs two lanes (host trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_graph_gpu.py tests/test_verify_mul_config.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 9; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/probes/vmhost.py > $O/vmhost.json 2> $O/vmhost.err || exit 1
SVDW_HOST_TRACE=1 timeout -k 10 300 python tools/probes/vmhost.py > $O/vmhost_t.json 2> $O/vmhost_trace.txt || exit 2
echo done
