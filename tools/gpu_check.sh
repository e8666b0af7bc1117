#!/bin/bash
# One GPU session: parity tests, smoke, bench, optional rocprofv3 kernel trace.
# Stops at the first step that faults / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${BENCH_N:-1024}
TAG=${TAG:-r01}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  if [ $rc -ge 2 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --n $N --steps ${STEPS:-10} --warmup 3 --breakdown > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --n $N --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
  rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_$TAG -name "*stats*" | head
fi
exit $rc
