#!/usr/bin/env python3
"""Time the virtual -> physical layout of the bench witness (1024^2, P=63):
plan (svdw_physical_layout, host) and svdw_assign_columns per phase (device
D2D column copies + selector bytes + lookup columns), with the bytes moved.

    python tools/probes/phys_time.py [--n 1024] [--p 63] [--k 24] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import gamma_for, gen_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--k", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import halo2_svd041_amd as hs
    m, u, d, v = gen_input(a.n, a.n, 0)
    dev = torch.device("cuda", 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)
                      for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(0))
    ctx.sync()
    t0 = time.perf_counter()
    p = ctx.physical_layout(a.k, 20)
    plan_ms = (time.perf_counter() - t0) * 1e3
    res = {"n": a.n, "P": a.p, "k": a.k, "plan_ms": round(plan_ms, 3), "params": p, "phases": {}}
    for ph in (0, 1):
        ctx.assign_columns(ph)                    # warm-up (allocations)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            adv, sel, lk = ctx.assign_columns(ph)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del adv, sel, lk
        t = min(ts)
        rows = 1 << a.k
        # read the virtual streams once, write every column in full (cells + q bytes)
        moved = ((ctx.advice_len(ph) + ctx.lookup_len(ph)) * 32 +
                 p["columns_used"][ph] * rows * 33 + p["num_lookup_advice"][ph] * rows * 32)
        res["phases"][ph] = {"ms": round(t * 1e3, 3), "bytes": moved,
                             "GB_per_s": round(moved / t / 1e9, 1)}
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
