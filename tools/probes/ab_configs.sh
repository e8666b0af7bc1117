#!/bin/bash
# Same-box A/B of libsvdw_base.so (tools/probes/build_base.sh) against the working
# tree's build at 1024^2 P=63, 512^2 P=32 and an 8-way shard rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
R=${ROUNDS:-3}
bash tools/probes/ab_lib.sh $R --no-check --no-profile || exit $?
bash tools/probes/ab_lib.sh $R --no-check --no-profile --n 512 --p 32 || exit $?
for i in $(seq 1 $R); do
  for v in base new; do
    if [ $v = base ]; then lib=$PWD/halo2_svd041_amd/libsvdw_base.so; else lib=$PWD/halo2_svd041_amd/libsvdw.so; fi
    SVDW_LIB=$lib timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 10 > gpurun_out/abs_$v.json 2>&1 || exit $?
    echo "shard8 $v $(grep -h step_ms gpurun_out/abs_$v.json | tr -d ' \n')"
  done
done
