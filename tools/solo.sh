#!/bin/bash
# Per-kernel durations with the streams serialised (overlap 0: each kernel has
# the chip to itself), 1024^2 P=63 and the 8-way shard's rank 0, from the
# engine's event profiler (bench.py --breakdown, all kernels).
#   bash tools/solo.sh tag [svdw options k=v ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
shift
O=gpurun_out/$T
mkdir -p $O
OPTS=""
for kv in "$@"; do OPTS="$OPTS --opt $kv"; done
timeout -k 10 240 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ingest --no-check --profile-prefix "" \
  --breakdown --opt overlap=0 --opt phase1_overlap=0 $OPTS > $O/solo.json 2> $O/solo.err || exit $?
python3 - "$O/solo.err" <<'EOF'
import json, sys
txt = open(sys.argv[1]).read()
i = txt.index('{')
d = json.loads(txt[i:txt.rindex('}') + 1])
for k, v in d["ms_per_step_by_kernel"].items():
    print(f"  solo {v * 1e3:9.1f} us  {k}")
EOF
