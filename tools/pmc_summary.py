#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into per-kernel HBM traffic.

    python tools/pmc_summary.py gpurun_out/pmc_r01d --config N=1024,M=1024,P=63,LB=19 \
        --out profiles/r01_pmc_summary.json

Per the MI355X guide (HBM section): FETCH_SIZE on gfx950 reports half the bytes
of wide coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for
16 B-per-lane streaming stores. Both are KiB in the CSV. traffic per launch =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024 / dispatches, per kernel name (template
arguments stripped).
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short(name):
    n = name.split("(")[0]
    for pre in ("void svdw::", "svdw::"):
        if n.startswith(pre):
            n = n[len(pre):]
    return n.split("<")[0]


def load(path, counter):
    per = defaultdict(lambda: [0, 0.0])
    f = os.path.join(path, "run_counter_collection.csv")
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            k = short(r["Kernel_Name"])
            per[k][0] += 1
            per[k][1] += float(r["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--config", default="")
    ap.add_argument("--out", required=True)
    ap.add_argument("--workload", default="svd")
    a = ap.parse_args()
    # the kernel sources the passes ran (written on the GPU box next to the
    # passes, tools/pmc.sh); bench.py only uses a summary of its own sources
    shaf = os.path.join(a.pmc_dir, "sources_sha16")
    if os.path.exists(shaf):
        sha = open(shaf).read().strip()
    else:
        from bench import sources_sha16
        sha = sources_sha16()
    fetch = load(os.path.join(a.pmc_dir, "pass1"), "FETCH_SIZE")
    write = load(os.path.join(a.pmc_dir, "pass2"), "WRITE_SIZE")
    cfg = dict(kv.split("=") for kv in a.config.split(",") if kv)
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({a.pmc_dir}), "
                     "bench.py --steps 2 --warmup 1 --no-profile",
           "correction": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH_SIZE halved on gfx950)",
           "config": {k: int(v) for k, v in cfg.items()},
           "workload": a.workload,
           "sources_sha16": sha,
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        nf, fk = fetch.get(k, [0, 0.0])
        nw, wk = write.get(k, [0, 0.0])
        n = max(nf, nw)
        if not n:
            continue
        fb, wb = 2 * fk * 1024 / max(nf, 1), wk * 1024 / max(nw, 1)
        out["kernels"][k] = {"dispatches": n, "read_bytes_per_launch": round(fb),
                             "write_bytes_per_launch": round(wb),
                             "traffic_per_launch": round(fb + wb)}
    # bench.py's event profiler aggregates every stage launch (k_stage and the
    # batched k_stage_multi) under "k_stage": the same aggregate per launch here
    parts = {k: v for k, v in out["kernels"].items() if k.startswith("k_stage")}
    if parts and "k_stage" not in parts or len(parts) > 1:
        n = sum(v["dispatches"] for v in parts.values())
        rd = sum(v["read_bytes_per_launch"] * v["dispatches"] for v in parts.values())
        wr = sum(v["write_bytes_per_launch"] * v["dispatches"] for v in parts.values())
        if "k_stage" in out["kernels"]:
            out["kernels"]["k_stage_single"] = out["kernels"].pop("k_stage")
        out["kernels"]["k_stage"] = {"dispatches": n, "read_bytes_per_launch": round(rd / n),
                                     "write_bytes_per_launch": round(wr / n),
                                     "traffic_per_launch": round((rd + wr) / n),
                                     "aggregate_of": sorted(parts)}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["traffic_per_launch"] * kv[1]["dispatches"]):
        print(f"{k:28s} x{v['dispatches']:4d}  read {v['read_bytes_per_launch'] / 1e6:10.2f} MB  "
              f"write {v['write_bytes_per_launch'] / 1e6:10.2f} MB per launch")


if __name__ == "__main__":
    main()
