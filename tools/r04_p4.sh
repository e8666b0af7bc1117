#!/bin/bash
# Round-4 probe: lanes after the stream_wait change; 8-way rank after the
# put_cell fix (A/B pipeline, steady-state trace); parity subset.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_parity_gpu.py -k "pipelined or sharded or products_on_cell" tests/test_graph_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 9; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/probes/vmhost.py > $O/vmhost.json 2> $O/vmhost.err || exit 1
: > $O/ab_s8.txt
for round in 1 2; do
  for v in "pipeline=1" "pipeline=0"; do
    for r in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $r --steps 20 --opt $v 2>>$O/ab.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 4
      echo "round $round s8 rank $r [$v] $ms" >> $O/ab_s8.txt
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ss_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 8 > /dev/null 2> $O/ss_s8.err || exit 3
echo done
