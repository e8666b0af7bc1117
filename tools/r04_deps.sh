#!/bin/bash
# dep_values after the flag-initialisation fix: the whole GPU suite with value
# dependencies as the default (SVDW_DEP_VALUES=1), then same-process A/B on the
# 8-way rank, 512^2, 1024^2 and config 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/deps4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest0.log 2>&1 || { tail -30 $O/pytest0.log; exit 1; }
tail -1 $O/pytest0.log
SVDW_DEP_VALUES=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.txt
for round in 1 2; do
  for v in "dep_values=1" "dep_values=0"; do
    for r in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $r --steps 20 --opt $v 2>>$O/ab.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 2
      echo "round $round s8 rank $r [$v] $ms" | tee -a $O/ab.txt
    done
  done
done
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 5 --variant on:dep_values=1 --variant off:dep_values=0 > $O/ab512.txt 2>>$O/ab.err || exit 3
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 3 --variant on:dep_values=1 --variant off:dep_values=0 > $O/ab1024.txt 2>>$O/ab.err || exit 3
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 3 --variant hi:stage_priority=1 --variant lo:stage_priority=0 > $O/ab1024_sp.txt 2>>$O/ab.err || exit 3
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline --opt dep_values=1 > $O/vm_on_$i.json 2>> $O/ab.err || exit 4
  timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline --opt dep_values=0 > $O/vm_off_$i.json 2>> $O/ab.err || exit 4
done
echo done
