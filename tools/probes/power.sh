#!/bin/bash
# Is the 1024^2 step power-limited? GPU power / clocks sampled while bench.py
# runs back-to-back witnesses (200 steps), and once idle.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${1:-gpurun_out/power}
mkdir -p $O
rocm-smi --showpower --showclocks > $O/idle.txt 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --no-ingest --no-profile --steps 12000 --warmup 3 > $O/bench.json 2> $O/bench.err &
P=$!
sleep 15
for i in 1 2 3 4 5 6 7 8; do rocm-smi --showpower --showclocks --showtemp > $O/busy_$i.txt 2>&1; sleep 2; done
wait $P
echo done
