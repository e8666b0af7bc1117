#!/bin/bash
# Round-6 evidence run, in two gpurun calls (each under the 20-minute limit):
#   PART=a  GPU suite + smoke, the PMC passes (FETCH_SIZE / WRITE_SIZE, one run
#           each) of every BASELINE workload, GPU-only timelines (hold_us) and a
#           steady-state trace;
#   then, locally, `python tools/evidence.py r06` writes their summaries into
#   profiles/ tagged with the kernel-source hash, and they are committed;
#   PART=b  the bench lines (which now find their own PMC traffic and, for
#           config 2, its GPU-only chain in profiles/), the rocprof kernel
#           stats of the bench, the shard simulation and the ingest timings.
# The kernel sources must not change between the two parts (bench.py refuses
# summaries of other sources). Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r06}
O=gpurun_out/final_$T
mkdir -p $O
export TMPDIR=/tmp
SHA=$(python3 -c "import bench; print(bench.sources_sha16())")
echo "$SHA" > $O/sources_sha16_${PART:-a}
NB="--no-cpu-baseline --no-profile --no-check --no-ingest"
if [ "${PART:-a}" = a ]; then
  echo "$SHA" > $O/sources_sha16
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
  tail -1 $O/smoke.log
  pmc() {   # pmc <name> <command...>: FETCH_SIZE and WRITE_SIZE passes, one run each
    local name=$1; shift
    mkdir -p $O/pmc_$name
    echo "$SHA" > $O/pmc_$name/sources_sha16
    local i=0
    for grp in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_$name/pass$i -o run -- "$@" > $O/pmc_${name}_pass$i.log 2>&1 || return 1
    done
  }
  pmc bench python3 bench.py --steps 2 --warmup 1 $NB || exit 3
  pmc s8 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 2 || exit 4
  pmc vm python3 bench.py --workload verify_mul --steps 2 --warmup 1 $NB || exit 5
  pmc 512 python3 bench.py --n 512 --p 32 --steps 2 --warmup 1 $NB || exit 6
  pmc 2048 python3 bench.py --n 2048 --m 1024 --p 32 --steps 2 --warmup 1 $NB || exit 7
  echo pmc ok
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_1024 -o run -- python3 bench.py --steps 5 --warmup 2 $NB --opt hold_us=3000 > /dev/null 2> $O/go_1024.err || exit 8
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_512 -o run -- python3 bench.py --n 512 --p 32 --steps 5 --warmup 2 $NB --opt hold_us=1500 > /dev/null 2> $O/go_512.err || exit 9
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 > /dev/null 2> $O/go_s8.err || exit 10
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_vm -o run -- python3 bench.py --workload verify_mul --steps 5 --warmup 2 $NB --opt hold_us=1000 > /dev/null 2> $O/go_vm.err || exit 11
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/steady_1024 -o run -- python3 bench.py --steps 12 --warmup 3 $NB > /dev/null 2> $O/steady_1024.err || exit 12
  echo part a done
  exit 0
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 14
head -c 300 $O/bench.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-check > $O/prof_bench.json 2> $O/prof_bench.err || exit 15
: > $O/configs.jsonl
for a in "--n 512 --p 32" "--n 2048 --m 1024 --p 32" "--workload verify_mul --steps 200 --warmup 20" "--n 4096 --p 63 --steps 3 --warmup 1 --no-cpu-baseline"; do
  timeout -k 10 600 python bench.py $a >> $O/configs.jsonl 2>> $O/configs.err || exit 16
done
echo configs ok
timeout -k 10 600 python tools/shard_sim.py --worlds 1,2,4,8 --steps 40 > $O/shard_sim.json 2> $O/shard_sim.err || exit 17
timeout -k 10 300 python tools/ingest_time.py > $O/ingest.jsonl 2> $O/ingest.err || exit 18
echo part b done
