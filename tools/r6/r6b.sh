#!/bin/bash
# Round-6 second GPU call: CRT GEMM probe with per-block timelines, the
# counter list and one SQ counter pass over the probe, a steady-state kernel
# trace of 512^2 P=32 with the profiler off (VERDICT r05 #4's 31 us hole), and
# bench.py lines with the profiler out of the timed steps.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 150 tools/probes/gemmprobe 1024 20 > $O/gemm.txt 2>&1
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc1 -o run -- tools/probes/gemmprobe 1024 3 quick > $O/pmc1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/b512 -o run -- python3 bench.py --n 512 --p 32 --steps 40 --warmup 3 --no-profile --no-check --no-ingest --no-cpu-baseline > $O/b512_trace.json 2> $O/b512_trace.err
python3 tools/steady.py "$(python3 -c "import glob,sys; print(sorted(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True))[0])" $O/b512)" --steps 5 > $O/steady_b512.txt 2>&1 || true
timeout -k 10 300 python3 bench.py --n 512 --p 32 --steps 40 > $O/b512.json 2> $O/b512.err
timeout -k 10 300 python3 bench.py > $O/b1024.json 2> $O/b1024.err
echo r6b done
