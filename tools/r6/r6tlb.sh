#!/bin/bash
# Round-6: UTCL1 translation counters of the stage kernels per allocation (realloc.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6tlb}
mkdir -p $O
export TMPDIR=/tmp
REALLOC_N=4 timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --kernel-trace --output-format csv -d $O/pmc -o run -- python3 tools/r6/realloc.py > $O/realloc.jsonl 2> $O/e.err
echo "rc $?"
echo r6tlb done
