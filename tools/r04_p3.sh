#!/bin/bash
# Round-4 probe: lanes vs two contexts under 4 / 8 hardware queues; the
# stage log (stream of each stage) of a pipelined 8-way rank step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/probes/vmhost.py > $O/vmhost_q4.json 2> $O/vmhost.err || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python tools/probes/vmhost.py > $O/vmhost_q8.json 2>> $O/vmhost.err || exit 2
SVDW_STAGE_LOG=1 timeout -k 10 200 python tools/shard_sim.py --worlds 8 --rank 0 --steps 2 > $O/s8.json 2> $O/s8_stagelog.txt || exit 3
echo done
