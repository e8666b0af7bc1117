#!/bin/bash
# Round-4 probe: pipelined phase 1 behind the diff on st2 (phase1_overlap 3)
# against st3 (auto), at 1024^2, 512^2 and the 8-way rank; parity of mode 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_parity_gpu.py -k "pipelined or tuning" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 9; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 --variant st3:phase1_overlap=1 --variant st2:phase1_overlap=3 > $O/ab1024.txt 2>>$O/ab.err || exit 3
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 8 --variant st3:phase1_overlap=1 --variant st2:phase1_overlap=3 > $O/ab512.txt 2>>$O/ab.err || exit 3
: > $O/ab_s8.txt
for round in 1 2; do
  for v in "phase1_overlap=1" "phase1_overlap=3"; do
    for r in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $r --steps 20 --opt $v 2>>$O/ab.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 4
      echo "round $round s8 rank $r [$v] $ms" >> $O/ab_s8.txt
    done
  done
done
echo done
