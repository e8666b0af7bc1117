set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/kp; mkdir -p $O; : > $O/kp.jsonl
for args in "--world 8 --rank 0" "--world 8 --rank 0 --opt bits_fold=0" "--world 8 --rank 0 --serial 0" "" "--opt bits_fold=0" "--n 512 --p 32"; do
  timeout -k 10 120 python tools/kprobe.py $args >> $O/kp.jsonl 2>>$O/kp.err || exit 1
done
