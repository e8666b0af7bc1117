#!/bin/bash
# (run on the CPU side: gpurun itself is the GPU call)
# gpurun with waits while the pod has no free slot (exit 3: nothing ran, nothing charged)
log=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
