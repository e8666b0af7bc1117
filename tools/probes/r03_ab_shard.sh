#!/bin/bash
# A/B of engine options on the 8-way row shard (ranks 0 and 5 timed alone,
# alternating variants, two rounds): bash tools/probes/r03_ab_shard.sh tag "opt=v opt=v" "opt=v" ...
# (an empty string is the default configuration)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=$1
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
: > $O/ab.txt
for round in 1 2; do
  for v in "$@"; do
    args=""
    for kv in $v; do args="$args --opt $kv"; done
    for r in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $r --steps 20 $args 2>>$O/ab.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 1
      echo "round $round rank $r [$v] $ms" | tee -a $O/ab.txt
    done
  done
done
