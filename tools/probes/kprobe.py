#!/usr/bin/env python3
"""Per-kernel durations of one svd_witness configuration with the streams
serialised (overlap 0, phase1_overlap 0): each kernel alone on the GPU.

    python tools/probes/kprobe.py [--n 1024] [--p 63] [--world 8 --rank 0] [--opt k=v ...]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import gamma_for, gen_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--serial", type=int, default=1)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    m, u, d, v = gen_input(a.n, a.n, 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device="cuda:0")
                      for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    if a.serial:
        ctx.set_option("overlap", 0)
        ctx.set_option("phase1_overlap", 0)
    for kv in a.opt:
        k, _, val = kv.partition("=")
        ctx.set_option(k, int(val))
    if a.world > 1:
        ctx.set_shard(a.rank, a.world)
    for i in range(3):
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(i))
    ctx.sync()
    ctx.profile(True, "")
    for i in range(a.steps):
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(10 + i))
    ctx.sync()
    st = ctx.profile_collect()
    ctx.close()
    out = sorted(((s["name"], s["launches"], round(s["total_ms"] / a.steps * 1e3, 1)) for s in st),
                 key=lambda x: -x[2])
    print(json.dumps({"n": a.n, "p": a.p, "world": a.world, "rank": a.rank, "opts": a.opt,
                      "us_per_step": out}))


if __name__ == "__main__":
    main()
