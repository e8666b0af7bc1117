#!/usr/bin/env python3
"""Block timeline of the CRT GEMM kernel (svdw_debug_trace): how many blocks
run at once, per-block durations, per-XCC and per-CU placement.

    python tools/gemm_trace.py --n 1024 [--rows 128] [--sym]
"""
import argparse
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import gen_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--sym", action="store_true")
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    from halo2_svd041_amd._lib import lib
    N = a.n
    m, u, d, v = gen_input(N, N, 0)
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    A = m[: a.rows] if a.rows else m
    za = hs.ZkMatrix.new(ctx, u if a.sym else A)
    zb = hs.ZkMatrix.new(ctx, v)
    b = za.transpose_matrix() if a.sym else zb.transpose_matrix()
    hs.honest_prover_mat_mul(ctx, za, b)
    ctx.sync()
    nb = 40 * ((N + 127) // 128) ** 2 + 64
    buf = torch.zeros(5 * nb, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    lib().svdw_debug_trace(buf.data_ptr())
    hs.honest_prover_mat_mul(ctx, za, b)
    ctx.sync()
    lib().svdw_debug_trace(None)
    t = buf.view(-1, 5).cpu().numpy().astype(np.uint64)
    t = t[t[:, 0] != 0]
    start = t[:, 0].astype(np.int64)
    pro = t[:, 1].astype(np.int64)
    loop = t[:, 2].astype(np.int64)
    end = t[:, 3].astype(np.int64)
    t = t[:, [0, 3, 4]]
    t0 = start.min()
    s_us = (start - t0) / 100.0
    e_us = (end - t0) / 100.0
    dur = e_us - s_us
    ev = sorted([(x, 1) for x in s_us] + [(x, -1) for x in e_us])
    cur = peak = 0
    area = 0.0
    last = 0.0
    for x, dlt in ev:
        area += cur * (x - last)
        last = x
        cur += dlt
        peak = max(peak, cur)
    span = e_us.max()
    xcc = (t[:, 2] >> np.uint64(32)).astype(np.int64)
    hw = (t[:, 2] & np.uint64(0xffffffff)).astype(np.int64)
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
    out = {"blocks": int(len(t)), "span_us": round(float(span), 2),
           "block_us": {"min": round(float(dur.min()), 2), "median": round(float(np.median(dur)), 2),
                        "max": round(float(dur.max()), 2)},
           "concurrency": {"avg": round(area / span, 1), "peak": peak},
           "phase_us_median": {"prologue": round(float(np.median(pro - start)) / 100, 2),
                               "k_loop": round(float(np.median(loop - pro)) / 100, 2),
                               "epilogue": round(float(np.median(end - loop)) / 100, 2)},
           "start_us_p50_p90_max": [round(float(np.percentile(s_us, q)), 2) for q in (50, 90, 100)],
           "per_xcc": dict(sorted(Counter(xcc.tolist()).items())),
           "distinct_cus": int(len(set(cu_key.tolist()))),
           "max_blocks_per_cu": int(max(Counter(cu_key.tolist()).values()))}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
