#!/bin/bash
# Round-6 A/B: the stage stream's first launch waits for the quantization (q_wait 1)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "pipelined or lifetime" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
V="--variant q0:q_wait=0 --variant q1:q_wait=1"
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 8 --steps 40 $V > $O/ab512.txt 2> $O/ab512.err
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 6 --steps 20 $V > $O/ab1024.txt 2> $O/ab1024.err
timeout -k 10 400 python3 tools/ab.py --n 2048 --m 1024 --p 32 --rounds 4 --steps 10 $V > $O/ab2048.txt 2> $O/ab2048.err
echo r6t done
