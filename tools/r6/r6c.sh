#!/bin/bash
# Round-6 third GPU call: the CRT GEMM kernels (gemm_kern 0-3) in the probe
# and in the step (tools/ab.py interleaved at 1024^2 P=63 and 512^2 P=32,
# shard_sim 8-way rank 0 per kernel), after their parity tests.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "tuning_options or held_inputs or gemm_kern" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 150 tools/probes/gemmprobe 1024 20 > $O/gemm.txt 2>&1
V="--variant k0:gemm_kern=0 --variant k1:gemm_kern=1 --variant k2:gemm_kern=2 --variant k3:gemm_kern=3 --variant k4:gemm_kern=4"
timeout -k 10 300 python3 tools/ab.py --n 1024 --p 63 --rounds 6 --steps 10 $V > $O/ab1024.txt 2> $O/ab1024.err
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 6 --steps 20 $V > $O/ab512.txt 2> $O/ab512.err
for r in 1 2; do for k in 0 1 2 4; do
  timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 --opt gemm_kern=$k > $O/s8_k${k}_$r.json 2>> $O/s8.err
done; done
echo r6c done
