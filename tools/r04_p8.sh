#!/bin/bash
# Round-4 probe: why bench.py 512^2 P=32 is slower than tools/ab.py (profiler,
# pipeline, stream priority).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p8
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --n 512 --p 32 --no-cpu-baseline --no-check --no-ingest"
: > $O/b512.txt
for v in "" "--no-profile" "--opt pipeline=0" "--opt gemm_priority=0" "--no-profile --opt pipeline=0" "--steps 30" ; do
  r=$(timeout -k 10 200 $B $v 2>>$O/err.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])") || exit 1
  echo "[$v] $r" >> $O/b512.txt
done
timeout -k 10 300 python tools/ab.py --n 512 --p 32 --rounds 3 --steps 10 --variant on:pipeline=1 --variant off:pipeline=0 --variant prof:prof=2 > $O/ab512.txt 2>>$O/err.txt || exit 2
echo done
