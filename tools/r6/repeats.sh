#!/bin/bash
# Round-6: default bench.py lines on the final sources (another box than the evidence run's)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-rep}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline >> $O/bench_repeats.jsonl 2>> $O/b.err
done
echo repeats done
