set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 3 --variant kc4: --variant kc1:gemm_kc=1 > gpurun_out/ab_kc_1024.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 5 --steps 5 --variant kc4: --variant kc1:gemm_kc=1 > gpurun_out/ab_kc_512.txt 2>&1 || exit $?
timeout -k 10 300 python tools/shard_sim.py --worlds 8 --steps 5 > gpurun_out/ss8_kc4.json 2>&1 || exit $?
timeout -k 10 300 python tools/shard_sim.py --worlds 8 --steps 5 --opt gemm_kc=1 > gpurun_out/ss8_kc1.json 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_kc_1024.txt gpurun_out/ab_kc_512.txt; grep -h step_ms gpurun_out/ss8_kc*.json
