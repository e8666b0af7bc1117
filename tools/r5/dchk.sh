#!/bin/bash
# round 5: pipelined placement of the d checks (dchk_at) and k_gamma_prep
# (gamma_at) -- parity, the 8-way rank (tools/shard_sim.py, alternating
# variants), then 1024^2 / 512^2 (tools/ab.py)
set -o pipefail
out=gpurun_out/${1:-r5p}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pipelined_witnesses or shard_rank_parity" > $out/pytest.log 2>&1 || exit $?
VARS=${VARS:-"base: g1:gamma_at=1 d1:dchk_at=1 d2:dchk_at=2 d1g1:dchk_at=1,gamma_at=1 d2g1:dchk_at=2,gamma_at=1"}
for r in 1 2; do
  for v in $VARS; do
    name=${v%%:*}; kvs=${v#*:}; args=""
    for kv in ${kvs//,/ }; do args="$args --opt $kv"; done
    timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 30 $args > $out/s8_${name}_$r.json 2>> $out/s8.err || exit $?
  done
done
V="--variant base: --variant d2g1:dchk_at=2,gamma_at=1 --variant d1g1:dchk_at=1,gamma_at=1"
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 $V > $out/ab1024.txt 2>&1 &&
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 10 $V > $out/ab512.txt 2>&1 || exit $?
echo dchk done
