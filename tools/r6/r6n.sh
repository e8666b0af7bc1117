#!/bin/bash
# Round-6: tools/r6/benchdiff.py (fresh vs fixed gamma, options set again or not)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r6n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/r6/benchdiff.py --n 512 --p 32 --steps 40 --rounds 5 > $O/diff512.txt 2> $O/diff.err
timeout -k 10 300 python3 tools/r6/benchdiff.py --n 1024 --p 63 --steps 10 --rounds 4 > $O/diff1024.txt 2>> $O/diff.err
echo r6n done
