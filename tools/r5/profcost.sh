#!/bin/bash
# round 5: cost of the event profiler in bench.py (stage launches recording
# their own events through their dispatch), profiler on / off alternating
set -o pipefail
out=gpurun_out/${1:-r5w}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "prof or bench or tuning" > $out/pytest.log 2>&1 || exit $?
B="--steps 20 --warmup 4 --no-cpu-baseline --no-ingest --no-check"
for r in 1 2 3; do
  for pf in "" "--no-profile"; do
    tag="p${pf:+off}_$r"
    timeout -k 10 120 python3 bench.py --n 512 --p 32 $B $pf > $out/n512_$tag.json 2> $out/n512_$tag.err || exit $?
    timeout -k 10 120 python3 bench.py $B $pf > $out/n1024_$tag.json 2> $out/n1024_$tag.err || exit $?
  done
done
echo profcost done
