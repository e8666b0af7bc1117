#!/bin/bash
# Round-6 diagnostic: GPU power / clocks / temperature sampled beside a long
# 1024^2 bench run (is the step power- or thermally-limited on slow boxes?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6p2}
mkdir -p $O
(rocm-smi --showpower --showclocks --showtemp > $O/smi_idle.txt 2>&1) || true
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 3 --no-check --no-ingest --no-cpu-baseline --no-profile > $O/bench.json 2> $O/bench.err &
B=$!
sleep 6
for i in 1 2 3; do (rocm-smi --showpower --showclocks --showtemp > $O/smi_run$i.txt 2>&1) || true; sleep 1; done
wait $B
echo "bench rc $?"
(rocm-smi --showpower --showclocks --showtemp > $O/smi_after.txt 2>&1) || true
echo r6p2 done
