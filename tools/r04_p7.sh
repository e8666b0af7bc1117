#!/bin/bash
# Round-4 probe: GPU suite + smoke with lanes on by default and the lazy
# side-stream wait; config 2 host probe and bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/p7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python tools/probes/vmhost.py > $O/vmhost.json 2> $O/vmhost.err || exit 3
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload verify_mul --no-cpu-baseline --warmup 8 > $O/vm_$i.json 2>> $O/vm.err || exit 4
done
echo done
