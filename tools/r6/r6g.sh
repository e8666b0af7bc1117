#!/bin/bash
# Round-6 seventh GPU call: steady-state kernel traces (profiler off) of 512^2
# P=32 with and without the stage stream's wait for the residue planes
# (res_wait), and bench.py lines of both, alternating.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6g}
mkdir -p $O
export TMPDIR=/tmp
for rw in 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t512_rw$rw -o run -- python3 bench.py --n 512 --p 32 --steps 40 --warmup 3 --no-profile --no-check --no-ingest --no-cpu-baseline --opt res_wait=$rw > $O/t512_rw$rw.json 2> $O/t512_rw$rw.err
  python3 tools/steady.py "$(python3 -c "import glob,sys; print(sorted(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True))[0])" $O/t512_rw$rw)" --steps 5 > $O/steady512_rw$rw.txt 2>&1 || true
done
for r in 1 2 3; do for rw in 1 0; do
  timeout -k 10 200 python3 bench.py --n 512 --p 32 --steps 40 --no-check --no-ingest --no-cpu-baseline --no-profile --opt res_wait=$rw > $O/b512_rw${rw}_$r.json 2>> $O/b.err
done; done
echo r6g done
