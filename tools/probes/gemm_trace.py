#!/usr/bin/env python3
"""Per-block timeline of the batched CRT GEMM (k_gemm_crt_multi) inside one
svd_witness: each block's start, end of its prologue (first barrier), end of
its K loop and end, on the 100 MHz wall clock (svdw_debug_trace).

    python tools/probes/gemm_trace.py [--n 1024] [--p 63] [--world 8 --rank 0] [--opt k=v ...]
"""
import argparse
import ctypes as ct
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
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    from halo2_svd041_amd import zk
    m, u, d, v = gen_input(a.n, a.n, 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device="cuda:0")
                      for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    for kv in a.opt:
        k, _, val = kv.partition("=")
        ctx.set_option(k, int(val))
    if a.world > 1:
        ctx.set_shard(a.rank, a.world)
    for i in range(3):
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(i))
    ctx.sync()
    nblk = 65536
    buf = torch.zeros(nblk * 5, dtype=torch.int64, device="cuda:0")
    zk.lib().svdw_debug_trace(ct.c_void_p(buf.data_ptr()))
    hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(99))
    ctx.sync()
    zk.lib().svdw_debug_trace(ct.c_void_p(0))
    t = buf.view(nblk, 5).cpu().numpy().astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    s, p1, p2, e = ((t[:, i] - t0) / 100.0 for i in range(4))    # us
    xcc = (t[:, 4] >> 32).astype(int)
    out = {"blocks": int(len(t)), "span_us": round(float(e.max()), 1),
           "prologue_us": [round(float(np.percentile(p1 - s, q)), 2) for q in (10, 50, 90)],
           "kloop_us": [round(float(np.percentile(p2 - p1, q)), 2) for q in (10, 50, 90)],
           "epilogue_us": [round(float(np.percentile(e - p2, q)), 2) for q in (10, 50, 90)],
           "block_us": [round(float(np.percentile(e - s, q)), 2) for q in (10, 50, 90)],
           "start_us": [round(float(np.percentile(s, q)), 1) for q in (0, 50, 100)],
           "per_xcc_blocks": np.bincount(xcc, minlength=8).tolist(),
           "concurrency_mean": round(float((e - s).sum() / max(e.max(), 1e-9)), 1),
           "n": a.n, "p": a.p, "world": a.world, "rank": a.rank, "opts": a.opt}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
