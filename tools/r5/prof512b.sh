#!/bin/bash
# round 5: cost of the profiler's start markers at 512^2 (SVDW_PROF_NOSTART: A/B only)
set -o pipefail
out=gpurun_out/${1:-r5ab}
mkdir -p $out
B="--n 512 --p 32 --steps 40 --warmup 5 --no-cpu-baseline --no-ingest --no-check"
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py $B --no-profile > $out/off_$r.json 2> $out/off_$r.err || exit $?
  timeout -k 10 120 python3 bench.py $B > $out/on_$r.json 2> $out/on_$r.err || exit $?
  SVDW_PROF_NOSTART=1 timeout -k 10 120 python3 bench.py $B > $out/nostart_$r.json 2> $out/nostart_$r.err || exit $?
done
echo prof512b done
