#!/bin/bash
# Round-4 probe: GPU suite + smoke, same-process A/B of q_aside (quantize beside
# the product chain) at 1024^2, 512^2 and the 8-way rank, config 2, GPU-only
# timelines, the GEMM's per-block trace, PMC write/fetch bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/q5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 3 --variant on:q_aside=1 --variant off:q_aside=0 > $O/ab1024.txt 2>>$O/ab.err || exit 3
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 5 --variant on:q_aside=1 --variant off:q_aside=0 > $O/ab512.txt 2>>$O/ab.err || exit 3
: > $O/ab_s8.txt
for round in 1 2; do
  for v in "q_aside=1" "q_aside=0"; do
    for r in 0 5; do
      ms=$(timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank $r --steps 20 --opt $v 2>>$O/ab.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 4
      echo "round $round s8 rank $r [$v] $ms" >> $O/ab_s8.txt
    done
  done
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline > $O/vm_$i.json 2>> $O/ab.err || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_1024 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest --opt hold_us=3000 > /dev/null 2> $O/go_1024.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 5 --opt hold_us=1500 > /dev/null 2> $O/go_s8.err || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_vm -o run -- python3 bench.py --workload verify_mul --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest --opt hold_us=1000 > /dev/null 2> $O/go_vm.err || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/go_512 -o run -- python3 bench.py --n 512 --p 32 --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-check --no-ingest --opt hold_us=1500 > /dev/null 2> $O/go_512.err || exit 9
for t in "" "--world 8 --rank 0" "--n 512 --p 32"; do
  timeout -k 10 200 python tools/probes/gemm_trace.py $t >> $O/gemm_trace.jsonl 2>> $O/ab.err || exit 11
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/pass$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-check --no-ingest > $O/pmc_pass$i.log 2>&1 || exit 10
done
echo done
