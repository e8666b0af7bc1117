#!/bin/bash
# GPU-only schedule of rank 0 of the 8-way shard with the streams serialised
# (overlap=0 phase1_overlap=0: each kernel has the chip to itself), next to the
# overlapped one: the sum of solo durations is the step's work, the overlapped
# span how well it packs.
#   bash tools/r03_solo8.sh tag [svdw options k=v ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
OPTS=""
for kv in "$@"; do OPTS="$OPTS --opt $kv"; done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/solo_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 --opt overlap=0 --opt phase1_overlap=0 $OPTS > /dev/null 2> $O/solo_s8.err || exit $?
f=$(ls $O/solo_s8/*/run_kernel_trace.csv 2>/dev/null | head -n 1)
[ -z "$f" ] && f=$(ls $O/solo_s8/run_kernel_trace.csv)
python3 tools/timeline.py "$f" --all > $O/solo_s8.timeline.txt || exit $?
cat $O/solo_s8.timeline.txt
