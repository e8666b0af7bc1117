#!/bin/bash
# Round-3 PMC passes, one counter group per pass (kernel trace only, no other
# tracing domains), each under its own kill timer: the 1-GPU bench (1024^2
# P=63) and rank 0 of the 8-way shard. Output under gpurun_out/pmc3/<run>/pass<k>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc3
mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/bench/pass$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-check --no-ingest > $O/bench_pass$i.log 2>&1
  rc=$?; echo "bench pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/bench_pass$i.log; exit $rc; }
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/s8/pass$i -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 2 > $O/s8_pass$i.log 2>&1
  rc=$?; echo "s8 pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/s8_pass$i.log; exit $rc; }
done
echo pmc done
