#!/bin/bash
# Round-4 probe: the CRT GEMM on a capped grid (SVDW_GEMM_GRID blocks looping over
# its tiles), so it holds fewer CUs beside the stage kernels; parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p15
mkdir -p $O
export TMPDIR=/tmp
SVDW_GEMM_GRID=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_parity_gpu.py -k "device_inputs or pipelined or full_size or sharded" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 9; }
tail -1 $O/pytest.log
: > $O/res.txt
for round in 1 2; do
  for g in 0 1024 512 256; do
    for a in "--n 512 --p 32" "--n 1024 --p 63"; do
      r=$(SVDW_GEMM_GRID=$g timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-check --no-ingest --no-profile --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
      echo "round $round grid $g [$a] $r" >> $O/res.txt
    done
    ms=$(SVDW_GEMM_GRID=$g timeout -k 10 120 python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 20 2>>$O/err.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['worlds']['8']['step_ms'])") || exit 2
    echo "round $round grid $g [s8 rank 0] $ms" >> $O/res.txt
  done
done
echo done
