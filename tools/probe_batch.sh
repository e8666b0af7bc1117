#!/bin/bash
# A/B of the stage batching (k_stage_multi) at the BASELINE shapes; GPU tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
V=${VARIANTS:-"--variant on: --variant off:stage_batch=0"}
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 3 $V > gpurun_out/ab_1024.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 5 $V > gpurun_out/ab_512.txt 2>&1 || exit $?
timeout -k 10 300 python tools/shard_sim.py --worlds 8 --steps 5 ${SS_A:-} > gpurun_out/ss8_a.json 2>&1 || exit $?
timeout -k 10 300 python tools/shard_sim.py --worlds 8 --steps 5 ${SS_B:---opt stage_batch=0} > gpurun_out/ss8_b.json 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_1024.txt gpurun_out/ab_512.txt | grep -v "^.*:   "; grep -h step_ms gpurun_out/ss8_a.json gpurun_out/ss8_b.json
