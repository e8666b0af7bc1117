#!/bin/bash
# Round-3 baseline on one box: shard simulation (1/2/4/8 ranks), GPU-only
# schedule of rank 0 of the 8-way shard and of rank 0 with the streams
# serialised (overlap off), and the 1-GPU bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
O=gpurun_out/r03
timeout -k 10 240 python3 tools/shard_sim.py --worlds 1,2,4,8 --steps 10 > $O/shard_sim.json 2> $O/shard_sim.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/go_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 > /dev/null 2> $O/go_s8.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/go_s8s -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 --opt phase1_overlap=0 --opt overlap=0 > /dev/null 2> $O/go_s8s.err || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
for d in go_s8 go_s8s; do
  f=$(ls $O/$d/*/run_kernel_trace.csv 2>/dev/null | head -n 1)
  [ -z "$f" ] && f=$(ls $O/$d/run_kernel_trace.csv)
  python3 tools/timeline.py "$f" --all > $O/$d.timeline.txt || exit $?
done
