#!/bin/bash
# One-wave quantize blocks: GPU tests, per-kernel probe, bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/quant
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/kp.jsonl
for args in "--world 8 --rank 0 --serial 0" "--serial 0" "--n 512 --p 32 --serial 0"; do
  timeout -k 10 120 python tools/kprobe.py $args >> $O/kp.jsonl 2>>$O/kp.err || exit 2
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit 3
timeout -k 10 300 python bench.py --n 512 --p 32 --no-cpu-baseline > $O/b512.json 2>>$O/bench.err || exit 3
timeout -k 10 300 python tools/shard_sim.py --worlds 8 --rank 0 --steps 20 > $O/s8r0.json 2>>$O/bench.err || exit 4
timeout -k 10 300 python tools/shard_sim.py --worlds 8 --rank 5 --steps 20 > $O/s8r5.json 2>>$O/bench.err || exit 4
