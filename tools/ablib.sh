#!/bin/bash
# Same-box A/B of two builds of libsvdw.so (SVDW_LIB): the in-tree build against
# ablib/libsvdw_base.so (an earlier commit's build), interleaved, bench.py
# without the profiler at 1024^2 and 512^2, shard_sim 8-way ranks 0 and 5.
#   bash tools/ablib.sh <out dir> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/ablib}
R=${2:-2}
mkdir -p $O
export TMPDIR=/tmp
: > $O/res.txt
for round in $(seq 1 $R); do
  for lib in new base; do
    if [ $lib = base ]; then export SVDW_LIB=$PWD/ablib/libsvdw_base.so; else unset SVDW_LIB; fi
    for a in "--n 512 --p 32" "--n 1024 --p 63"; do
      r=$(timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-check --no-ingest --no-profile --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
      echo "round $round $lib [$a] $r" >> $O/res.txt
    done
    for rk in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $rk --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 2
      echo "round $round $lib [s8 rank $rk] $ms" >> $O/res.txt
    done
  done
done
unset SVDW_LIB
echo done
