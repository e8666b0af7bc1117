#!/bin/bash
# Round-6 sixth GPU call: four terms per row-scan thread (scan_t 4) against
# two, in the step and with the streams serialised (the scans' standalone
# time), at 1024^2 P=63 and 512^2 P=32, plus the 8-way shard rank.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
V="--variant base: --variant st4:scan_t=4 --variant rw0:res_wait=0 --variant rw0st4:res_wait=0,scan_t=4 --variant ser:overlap=0,phase1_overlap=0,pipeline=0 --variant ser4:overlap=0,phase1_overlap=0,pipeline=0,scan_t=4"
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 5 --steps 10 --top 14 $V > $O/ab1024.txt 2> $O/ab1024.err
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 5 --steps 20 --top 14 $V > $O/ab512.txt 2> $O/ab512.err
for r in 1 2; do for o in "scan_t=2" "scan_t=4" "res_wait=0"; do
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 --opt $o > $O/s8_${o}_$r.json 2>> $O/s8.err
done; done
echo r6f done
