#!/bin/bash
# steady-state kernel traces (no hold) of the 8-way rank and of 512^2 P=32
set -o pipefail
out=gpurun_out/${1:-r5s}
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/s8 -o run -- python3 tools/shard_sim.py --worlds 8 --rank 0 --steps 30 > $out/s8.json 2> $out/s8.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/b512 -o run -- python3 bench.py --n 512 --p 32 --steps 20 --warmup 3 > $out/b512.json 2> $out/b512.err || exit $?
echo steady done
