#!/usr/bin/env python3
"""Per-kernel table from `bench.py --breakdown` stderr (JSON after any noise).

    python tools/breakdown.py gpurun_out/bd.err [--steps K]
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    t = open(a.file).read()
    d = json.loads(t[t.index("{"):])
    tot = 0.0
    for k in sorted(d["stats"], key=lambda r: -r["total_ms"]):
        ms = k["total_ms"] / a.steps
        tot += ms
        bw = k["bytes"] / a.steps / (ms * 1e-3) / 1e12 if ms > 0 and k["bytes"] else 0.0
        print(f"{k['name']:44s} {ms * 1e3:8.1f} us/step  x{k['launches'] / a.steps:4.1f}  {bw:5.2f} TB/s")
    print(f"{'sum':44s} {tot * 1e3:8.1f} us/step")


if __name__ == "__main__":
    main()
