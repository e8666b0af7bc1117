#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, no tracing
# domains besides the kernel trace, per the pool's rules). Output under
# gpurun_out/pmc_<TAG>/pass<k>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
N=${BENCH_N:-1024}
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
mkdir -p gpurun_out/pmc_$TAG
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/pass$i -o run -- python3 bench.py --n $N --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-check > gpurun_out/pmc_$TAG/pass$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$TAG/pass$i.log; exit $rc; fi
done
