#!/bin/bash
# round 5: stream priorities (SVDW_PRIO: cell stream, st2, st3) with 256- and
# XCD-contiguous 64-element stage blocks; bench.py processes, alternating
set -o pipefail
out=gpurun_out/${1:-r5v}
mkdir -p $out
B="--steps 20 --warmup 4 --no-cpu-baseline --no-ingest --no-profile --no-check"
python3 -c "import torch,ctypes; h=ctypes.CDLL('libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); print('prio range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)), a.value, b.value)" > $out/range.txt 2>&1
for r in 1 2; do
  for pr in "" "0,0,-1" "-1,0,-1" "0,1,0"; do
    for el in 256 64; do
      tag="p${pr//,/_}_e${el}_$r"
      X=""; [ $el = 64 ] && X="--opt stage_elems=64 --opt stage_xcd=1"
      SVDW_PRIO="$pr" timeout -k 10 120 python3 bench.py $B $X > $out/$tag.json 2> $out/$tag.err || exit $?
      SVDW_PRIO="$pr" timeout -k 10 120 python3 bench.py --n 512 --p 32 $B $X > $out/n512_$tag.json 2> $out/n512_$tag.err || exit $?
    done
  done
done
echo prio done
