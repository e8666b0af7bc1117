#!/bin/bash
# Round-4 probe: GPU suite + smoke after the pipelined d-check move; A/B of
# pipeline at 1024^2, 512^2 and the 8-way rank; steady-state 8-way trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
: > $O/ab_s8.txt
for round in 1 2; do
  for v in "pipeline=1" "pipeline=0"; do
    for r in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $r --steps 20 --opt $v 2>>$O/ab.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 4
      echo "round $round s8 rank $r [$v] $ms" >> $O/ab_s8.txt
    done
  done
done
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 --variant on:pipeline=1 --variant off:pipeline=0 > $O/ab1024.txt 2>>$O/ab.err || exit 3
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 8 --variant on:pipeline=1 --variant off:pipeline=0 > $O/ab512.txt 2>>$O/ab.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ss_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 8 > /dev/null 2> $O/ss_s8.err || exit 5
echo done
SVDW_HOST_TRACE=1 timeout -k 10 200 python tools/probes/vmhost.py > $O/vmhost.json 2> $O/vmhost_trace.txt || exit 6
echo done2
