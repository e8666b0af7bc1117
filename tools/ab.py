#!/usr/bin/env python3
"""Interleaved A/B of engine tuning options in ONE process (guide rule 24).

    python tools/ab.py --n 1024 --p 63 --rounds 5 --steps 3 \
        --variant base: --variant e64:stage_elems=64 --variant p1:phase1_overlap=2
Prints median / min ms per step and per-kernel medians for each variant.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import gamma_for, gen_input  # noqa: E402


def parse_variant(s):
    name, _, rest = s.partition(":")
    opts = {}
    for kv in filter(None, rest.split(",")):
        k, v = kv.split("=")
        opts[k] = int(v)
    return name, opts


# every option a variant may set, at its engine default (variants share one
# context, so an option left out here would leak from one variant into the next)
DEFAULTS = {"gemm_impl": 0, "overlap": 1, "gemm_crt": 1, "stage_elems": 256,
            "phase1_overlap": 1, "p1_at": -1, "prod_cell": 1, "res_f64": 1,
            "stage_batch": 1, "f64_views": 1, "pipeline": 1, "vm_linear": 1,
            "dchk_at": 0, "gamma_at": -1, "gemm_kern": -1, "res_wait": -1, "stage_rot": 1, "place_trials": 6}
# pseudo-option "prof": event profiler during the timed steps (0 off, 1 all, 2 k_stage only)
PROF_PREFIX = {1: "", 2: "k_stage"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--top", type=int, default=8, help="kernels listed per variant")
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    N, M = a.n, a.m or a.n
    m, u, d, v = gen_input(N, M, 0)
    g = gamma_for(0)
    dev = torch.device("cuda", 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    variants = [parse_variant(s) for s in (a.variant or ["base:"])]
    res = {name: [] for name, _ in variants}
    kern = {name: {} for name, _ in variants}
    for name, opts in variants:          # warm every variant once
        for k, val in {**DEFAULTS, **opts}.items():
            if k != "prof":
                ctx.set_option(k, val)
        hs.svd_witness(ctx, dm, du, dv, dd, g)
    ctx.sync()
    for _ in range(a.rounds):
        for name, opts in variants:
            prof = opts.get("prof", 0)
            for k, val in {**DEFAULTS, **opts}.items():
                if k != "prof":
                    ctx.set_option(k, val)
            hs.svd_witness(ctx, dm, du, dv, dd, g)
            ctx.sync()
            if prof:
                ctx.profile(True, PROF_PREFIX[prof])
            t0 = time.perf_counter()
            for _ in range(a.steps):
                hs.svd_witness(ctx, dm, du, dv, dd, g)
            ctx.sync()
            res[name].append((time.perf_counter() - t0) / a.steps * 1e3)
            if prof:
                ctx.profile_collect()
                ctx.profile(False)
            ctx.profile(True)
            hs.svd_witness(ctx, dm, du, dv, dd, g)
            for s in ctx.profile_collect():
                kern[name].setdefault(s["name"], []).append(s["total_ms"])
            ctx.profile(False)
    cells = sum(hs.plan_svd(N, M, a.p, 19)[k] for k in ("advice0", "advice1"))
    for name, _ in variants:
        med = statistics.median(res[name])
        print(f"{name:12s} median {med:.4f} ms  min {min(res[name]):.4f}  -> {cells / med / 1e6:.2f} Gcells/s"
              f"  samples {' '.join(f'{x:.3f}' for x in sorted(res[name]))}"
              f"  (in order {' '.join(f'{x:.3f}' for x in res[name])})")
        top = sorted(kern[name].items(), key=lambda kv: -statistics.median(kv[1]))[:a.top]
        print("   " + "  ".join(f"{k}={statistics.median(vv):.3f}" for k, vv in top))
    print(json.dumps({n: statistics.median(r) for n, r in res.items()}))


if __name__ == "__main__":
    main()
