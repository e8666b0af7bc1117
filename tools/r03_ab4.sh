set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ab.py --n 1024 --p 63 --rounds 5 --steps 5 --variant base: --variant pf:prod_first=1 --variant pcpf:prod_cell=1,prod_first=1 --variant gp:gemm_priority=1,prod_first=1 > gpurun_out/ab4/ab1024.txt 2>&1 || exit 1
tail -9 gpurun_out/ab4/ab1024.txt
