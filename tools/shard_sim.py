#!/usr/bin/env python3
"""One GPU standing in for each rank of a row-sharded witness (BASELINE config 4).

    python tools/shard_sim.py --n 1024 --p 63 --worlds 1,2,4,8 --steps 5

For every world size W and rank r, a context with svdw_set_shard(r, W) runs the
witness (its own row blocks, plus the inputs every rank recomputes) and is
timed alone; the slowest rank is the strong-scaling step time of a W-GPU node
with the witness kept sharded-resident (no reassembly, no interconnect). The
whole-job rate is the one-matrix advice cells / that time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import gamma_for, gen_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rank", type=int, default=None, help="time only this rank of each world")
    ap.add_argument("--opt", action="append", default=[], help="svdw_set_option name=value")
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    N, M = a.n, a.m or a.n
    m, u, d, v = gen_input(N, M, 0)
    g = gamma_for(0)
    dev = torch.device("cuda", 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)
                      for x in (m, u, v, d))
    cells = None
    res = {}
    for W in [int(w) for w in a.worlds.split(",")]:
        per_rank = []
        for r in (range(W) if a.rank is None else [a.rank % W]):
            ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
            for kv in a.opt:
                k, _, val = kv.partition("=")
                ctx.set_option(k, int(val))
            if W > 1:
                ctx.set_shard(r, W)
            cnt = hs.svd_witness(ctx, dm, du, dv, dd, g)   # warm-up
            hs.svd_witness(ctx, dm, du, dv, dd, g)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                hs.svd_witness(ctx, dm, du, dv, dd, g)
            ctx.sync()
            per_rank.append((time.perf_counter() - t0) / a.steps)
            ctx.close()
            cells = cnt["advice0"] + cnt["advice1"]
        t = max(per_rank)
        res[W] = {"step_ms": round(t * 1e3, 4), "rank_ms": [round(x * 1e3, 3) for x in per_rank],
                  "advice_cells_per_s": round(cells / t, 1)}
    t1 = res.get(1, {}).get("step_ms")
    for W, r in res.items():
        if t1:
            r["efficiency_vs_1"] = round(t1 / (W * r["step_ms"]), 4)
    print(json.dumps({"N": N, "M": M, "P": a.p, "worlds": res}, indent=1))


if __name__ == "__main__":
    main()
