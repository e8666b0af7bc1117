#!/bin/bash
# same-box A/B of the round-4 head (f6f5b89, tree in ablib/r4)
# against the round-5 head (35a327a, tree in ablib/r5), each with its own
# bench.py, shard_sim.py and libsvdw.so, runs alternating; bench without the
# event profiler, 20 steps: 1024^2 P=63, 512^2 P=32, 8-way shard rank 0.
#   bash tools/r6/ab45.sh <out dir> [rounds]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/${1:-gpurun_out/ab45}
R=${2:-3}
mkdir -p $O
export TMPDIR=/tmp
: > $O/res.txt
for round in $(seq 1 $R); do
  for t in r4 r5; do
    cd $ROOT/ablib/$t
    for a in "--n 1024 --p 63" "--n 512 --p 32"; do
      r=$(timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-check --no-ingest --no-profile --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
      echo "round $round $t [$a] $r" | tee -a $O/res.txt
    done
    ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 2
    echo "round $round $t [s8 rank 0] $ms" | tee -a $O/res.txt
  done
done
echo done
