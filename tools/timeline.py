#!/usr/bin/env python3
"""Per-step timeline from a rocprofv3 kernel trace (run_kernel_trace.csv).

    python tools/timeline.py gpurun_out/prof_X/run_kernel_trace.csv [--steps 5]

Splits the trace into witness steps (each starts with the first k_quantize of
the step), then for the last step prints every dispatch (stream, start offset,
duration, grid) and the busy / idle time of the union of all streams, so
launch gaps and serial tails are visible.
"""
import argparse
import csv
import json
import os
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for pre in ("void svdw::", "svdw::"):
        if n.startswith(pre):
            n = n[len(pre):]
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--all", action="store_true", help="print every dispatch of the last step")
    ap.add_argument("--json", default=None, help="also write the step summary and its critical chain here")
    ap.add_argument("--workload", default=None, help="workload tag recorded in --json (e.g. verify_mul)")
    ap.add_argument("--sha", default=None, help="kernel-source hash recorded in --json (bench.sources_sha16)")
    ap.add_argument("--config", default="", help="N=..,M=..,P=..,LB=.. recorded in --json")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Stream_Id", r.get("Queue_Id")), int(r["Grid_Size_X"])))
    rows.sort()
    # step boundaries: with hold_us, each k_hold ends where a step's queued
    # work starts; else the first k_bits_f64 / k_quantize of a run of them
    holds = [i for i, r in enumerate(rows) if r[2].startswith("k_hold")]
    if len(holds) >= 2:
        h0, h1 = holds[-2], holds[-1]
        step = [r for r in rows if rows[h0][1] <= r[0] < rows[h1][1] and not r[2].startswith("k_hold")]
        step_end = max(r[1] for r in step)           # (the next step waits behind its hold)
    else:
        mark = lambda n: n.startswith("k_quantize") or n.startswith("k_bits_f64")   # noqa: E731
        starts = [i for i, r in enumerate(rows) if mark(r[2]) and (i == 0 or not mark(rows[i - 1][2]))]
        if len(starts) < 2:
            raise SystemExit("could not find step boundaries")
        s0, s1 = starts[-2], starts[-1]
        step = rows[s0:s1]
        step_end = rows[s1][0]
    t0 = step[0][0]
    tend = max(r[1] for r in step)
    span = (step_end - t0) / 1e3
    # union busy time
    busy, cur_s, cur_e = 0, None, None
    for s, e, *_ in step:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"step span (start to next step start) {span:.1f} us, last kernel end {(tend - t0) / 1e3:.1f} us, "
          f"GPU busy (union) {busy / 1e3:.1f} us, idle {span - busy / 1e3:.1f} us, dispatches {len(step)}")
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, n, st, g in step:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
    for n, (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {tot:9.1f} us  x{cnt:3d}  {n}")
    # critical chain: back from the last kernel to end, each time to the kernel
    # (any stream) that ended last before the current one started -- what it
    # waited for in a GPU-only (hold_us) schedule; boundary = the gaps between
    chain = [max(step, key=lambda r: r[1])]
    while True:
        cur = chain[-1]
        prev = [r for r in step if r[1] <= cur[0] and r is not cur]
        if not prev:
            break
        chain.append(max(prev, key=lambda r: r[1]))
    chain.reverse()
    kern = sum(r[1] - r[0] for r in chain) / 1e3
    gaps = sum(max(0, chain[i + 1][0] - chain[i][1]) for i in range(len(chain) - 1)) / 1e3
    lead = (chain[0][0] - t0) / 1e3
    print(f"critical chain: {len(chain)} launches, {kern:.1f} us in kernels, {gaps:.1f} us at launch "
          f"boundaries, starts {lead:.1f} us into the step: " + " -> ".join(r[2] for r in chain))
    if a.json:
        out = {"span_us": round(span, 1), "busy_us": round(busy / 1e3, 1), "dispatches": len(step),
               "chain": {"launches": len(chain), "kernel_us": round(kern, 1), "boundary_us": round(gaps, 1),
                         "lead_us": round(lead, 1), "kernels": [r[2] for r in chain]},
               "kernels_us": {n: round(t, 1) for n, (c, t) in agg.items()},
               "source": os.path.relpath(a.trace), "workload": a.workload, "sources_sha16": a.sha,
               "config": {k: int(v) for k, v in (kv.split("=") for kv in a.config.split(",") if kv)}}
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)
    if a.all:
        prev_end = t0
        for s, e, n, st, g in step:
            print(f"  s{st} +{(s - t0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f} gap {(s - prev_end) / 1e3:6.1f} "
                  f"grid {g:9d}  {n}")
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
