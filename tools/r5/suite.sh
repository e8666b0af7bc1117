#!/bin/bash
# the GPU suite, then the simulated strong scaling of config 4 (tools/shard_sim.py)
set -o pipefail
out=gpurun_out/${1:-r5r}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $out/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/shard_sim.py --worlds 1,2,4,8 --steps 20 > $out/shard_sim.json 2> $out/shard_sim.err || exit $?
echo suite done
