#!/usr/bin/env python3
"""Per-kernel averages of every counter in the PMC passes of tools/pmc.sh.

    python tools/pmc_kernel.py gpurun_out/pmc_r01d [kernel-substring ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for pre in ("void svdw::", "svdw::"):
        if n.startswith(pre):
            n = n[len(pre):]
    return n


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    agg = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for f in sorted(glob.glob(os.path.join(d, "pass*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if want and not any(w in k for w in want):
                    continue
                a = agg[k][r["Counter_Name"]]
                a[0] += 1
                a[1] += float(r["Counter_Value"])
    for k, cs in sorted(agg.items()):
        print(k)
        for c, (n, v) in sorted(cs.items()):
            print(f"   {c:24s} avg {v / n:16.1f}   (n={n})")


if __name__ == "__main__":
    main()
