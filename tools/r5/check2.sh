#!/bin/bash
# round 5: full GPU suite, a default bench line, config-2 bench, small_spread A/B (1024^2, 512^2, 8-way rank)
set -o pipefail
out=gpurun_out/${1:-r5i}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || exit 3
timeout -k 10 300 python bench.py --workload verify_mul > $out/vm.json 2> $out/vm.err || exit 4
V="--variant sp1:small_spread=1 --variant sp0:small_spread=0" S8=1 ./tools/r5/ab2.sh ${1:-r5i}
