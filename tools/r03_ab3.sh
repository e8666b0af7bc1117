set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3
timeout -k 10 120 ./tools/wtgap > gpurun_out/ab3/wtgap.txt 2>&1 || exit 1
cat gpurun_out/ab3/wtgap.txt
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "full_size" > gpurun_out/ab3/pytest.log 2>&1 || { tail -30 gpurun_out/ab3/pytest.log; exit 1; }
tail -2 gpurun_out/ab3/pytest.log
timeout -k 10 300 python3 tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 --variant base: --variant pf:prod_first=1 --variant pc:prod_cell=1 --variant pcpf:prod_cell=1,prod_first=1 > gpurun_out/ab3/ab1024.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab.py --n 512 --p 32 --rounds 5 --steps 5 --variant base: --variant pf:prod_first=1 --variant pc:prod_cell=1 > gpurun_out/ab3/ab512.txt 2>&1 || exit 1
bash tools/r03_ab_shard.sh ab3s "" "res_first=0" "prod_first=1" "stage_priority=1"
