#!/usr/bin/env python3
"""Steady-state view of pipelined witnesses from a rocprofv3 kernel trace (no
hold_us): step span between consecutive k_quantize starts, per-stream kernel
time per step (which stream is saturated), and one step's dispatches.

    python tools/steady.py gpurun_out/x/run_kernel_trace.csv [--steps 3]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void svdw::", "").replace("svdw::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:30],
                         r.get("Stream_Id", r.get("Queue_Id")), int(r["Grid_Size_X"])))
    rows.sort()
    qs = [i for i, r in enumerate(rows) if r[2].startswith("k_quantize")]
    if len(qs) < a.steps + 2:
        raise SystemExit("trace too short")
    i0, i1 = qs[-(a.steps + 2)], qs[-2]
    span = (rows[i1][0] - rows[i0][0]) / 1e3 / a.steps
    load = collections.defaultdict(float)
    for r in rows[i0:i1]:
        load[r[3]] += (r[1] - r[0]) / 1e3
    print(f"steady state over {a.steps} steps: {span:.1f} us per step")
    print("kernel time per step by stream: " +
          ", ".join(f"stream {k}: {v / a.steps:.1f} us" for k, v in sorted(load.items())))
    t0 = rows[qs[-3]][0]
    print("one step (offsets from its k_quantize start; other streams still run the previous call):")
    for r in rows[qs[-3]:qs[-2]]:
        print(f"  stream {r[3]:>3} +{(r[0] - t0) / 1e3:8.1f} us  dur {(r[1] - r[0]) / 1e3:7.1f} us  "
              f"grid {r[4]:8d}  {r[2]}")


if __name__ == "__main__":
    main()
