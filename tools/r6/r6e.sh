#!/bin/bash
# Round-6 fifth GPU call: wave priority of the product chain (chain_prio:
# quantize, residues, GEMM, combine) with the shipped / persistent / LDS-DMA
# GEMM, interleaved at 512^2 P=32, 1024^2 P=63 and on the 8-way shard rank.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
V="--variant base: --variant cp1:chain_prio=1 --variant cp3:chain_prio=3 --variant cp3k4:chain_prio=3,gemm_kern=4 --variant cp3k2:chain_prio=3,gemm_kern=2 --variant k4:gemm_kern=4"
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 6 --steps 20 $V > $O/ab512.txt 2> $O/ab512.err
timeout -k 10 400 python3 tools/ab.py --n 1024 --p 63 --rounds 5 --steps 10 $V > $O/ab1024.txt 2> $O/ab1024.err
for r in 1 2; do for o in "chain_prio=0" "chain_prio=3" "chain_prio=3 --opt gemm_kern=4" "chain_prio=1"; do
  n=$(echo $o | tr -c 'a-z0-9' '_')
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 --opt $o > $O/s8_${n}_$r.json 2>> $O/s8.err
done; done
echo r6e done
