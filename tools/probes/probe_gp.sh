#!/bin/bash
# gemm_priority (high-priority product stream) across witness shapes (tools/ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "--n 256 --p 32" "--n 512 --p 63" "--n 768 --p 63" "--n 1024 --p 63" "--n 1024 --p 32" "--n 2048 --m 1024 --p 32"; do
  timeout -k 10 300 python tools/ab.py $s --rounds ${R:-4} --steps 6 --variant base: --variant gp:gemm_priority=1 > gpurun_out/abgp.txt 2>&1 || exit $?
  echo "$s $(tail -1 gpurun_out/abgp.txt)"
done
