#!/bin/bash
# GEMM standalone timings + one PMC pass on the non-symmetric 1024^2 product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-gemm}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for args in "--n 1024" "--n 1024 --sym" "--n 1024 --rows 128"; do
  timeout -k 10 120 python3 tools/gemm_bench.py $args >> $O/gemm.jsonl 2>> $O/gemm.err || exit $?
done
cat $O/gemm.jsonl
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 tools/gemm_bench.py --n 1024 --reps 3 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/pmc2 -o run -- python3 tools/gemm_bench.py --n 1024 --reps 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    if "gemm" not in k and "combine" not in k and "residues" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
