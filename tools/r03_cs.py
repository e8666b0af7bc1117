#!/usr/bin/env python3
"""Per-kernel times of the 8-way shard's rank 0 (engine event profiler) with
the given options, and the is_equal rows' z cells (all 1 for an honest witness).

    python tools/r03_cs.py [--opt k=v ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import gamma_for, gen_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    N = 1024
    m, u, d, v = gen_input(N, N, 0)
    g = gamma_for(0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device="cuda")
                      for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=63, lookup_bits=19)
    for kv in a.opt:
        k, _, val = kv.partition("=")
        ctx.set_option(k, int(val))
    if a.world > 1:
        ctx.set_shard(0, a.world)
    hs.svd_witness(ctx, dm, du, dv, dd, g)
    ctx.sync()
    ctx.profile(True, "")
    for _ in range(3):
        hs.svd_witness(ctx, dm, du, dv, dd, g)
    st = ctx.profile_collect()
    ctx.profile(False)
    out = {s["name"]: round(s["total_ms"] / s["launches"] * 1e3, 1) for s in st}
    zs = []
    for r in ctx.layout():
        if "is_equal" in r["tag"]:
            cells = ctx.advice(r["phase"], r["off"], min(r["n"], 12 * 128))
            z = cells.reshape(-1, 12, cells.shape[-1])[:, 4]
            zs.append(int((z[:, 0] == 1).sum()))
    print(json.dumps({"opts": a.opt, "kernels_us": out, "z_ones_first128": zs}))
    ctx.close()


if __name__ == "__main__":
    main()
