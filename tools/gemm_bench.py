#!/usr/bin/env python3
"""Standalone timing of the exact field GEMM (honest_prover_mat_mul through the
ABI: residue planes from the cells, the multi-modular int8 MFMA GEMM, the CRT
combine), per kernel from the engine's event profiler.

    python tools/gemm_bench.py --n 1024 --p 63 --reps 10 [--sym]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import gen_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=None, help="rows of A (a row block)")
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sym", action="store_true", help="u . u^T (upper tiles + mirror)")
    ap.add_argument("--opt", action="append", default=[], help="svdw_set_option name=value")
    a = ap.parse_args()
    import halo2_svd041_amd as hs
    N = a.n
    m, u, d, v = gen_input(N, N, 0)
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    for kv in a.opt:
        k, _, val = kv.partition("=")
        ctx.set_option(k, int(val))
    A = m[: a.rows] if a.rows else m
    za = hs.ZkMatrix.new(ctx, u if a.sym else A)
    zb = hs.ZkMatrix.new(ctx, v)
    b = za.transpose_matrix() if a.sym else zb.transpose_matrix()
    hs.honest_prover_mat_mul(ctx, za, b)                  # warm-up (and the bound reads)
    ctx.sync()
    ctx.profile(True, "")
    for _ in range(a.reps):
        hs.honest_prover_mat_mul(ctx, za, b)
    stats = ctx.profile_collect()
    ctx.profile(False)
    rows = za.num_rows
    macs = float(rows) * N * N
    out = {"N": N, "rows": rows, "P": a.p, "sym": a.sym, "opts": a.opt, "kernels": {}}
    tot = 0.0
    for s in stats:
        ms = s["total_ms"] / s["launches"]
        tot += ms
        out["kernels"][s["name"]] = round(ms * 1e3, 2)
    out["total_us"] = round(tot * 1e3, 2)
    out["field_GMAC_s"] = round(macs / (tot * 1e-3) / 1e9, 1)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
