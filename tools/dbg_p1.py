"""Debug aid: witness vs C oracle per (shape, option set); prints the layout
regions whose cells differ (first few) for each phase.

    python tools/dbg_p1.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import corc  # noqa: E402
import halo2_svd041_amd as hs  # noqa: E402
from conftest import gamma_for, gen_svd_input  # noqa: E402

SHAPES = [(4, 4, 32), (6, 5, 63), (5, 7, 42), (24, 20, 63), (64, 64, 63)]
OPTS = [{}, {"scan_na_host": 1}, {"phase1_overlap": 0}, {"scan_impl": 3}, {"scan_impl": 4}]


def diff_regions(ctx, phase, got, want):
    bad = np.nonzero(np.any(got != want, axis=1))[0] if got.shape == want.shape else None
    if bad is None:
        return f"shape {got.shape} vs {want.shape}"
    if not len(bad):
        return "ok"
    out = []
    for r in ctx.layout():
        if r["phase"] != phase:
            continue
        k = np.count_nonzero((bad >= r["off"]) & (bad < r["off"] + r["n"]))
        if k:
            out.append(f"{r['tag']}@{r['off']}+{r['n']}:{k}")
    return f"{len(bad)} bad: " + " ".join(out[:8])


for N, M, P in SHAPES:
    m, u, d, v = gen_svd_input(N, M, seed=N * 7 + M + P)
    g = gamma_for(P)
    a0, l0, a1 = corc.svd_witness(m, u, v, d, P, 19, g)
    for o in OPTS:
        with hs.Context(device=0, precision_bits=P, lookup_bits=19) as ctx:
            for k, val in o.items():
                ctx.set_option(k, val)
            hs.svd_witness(ctx, m, u, v, d, g)
            ctx.sync()
            print(f"{N}x{M} P={P} {o}: ph0 {diff_regions(ctx, 0, ctx.advice(0), a0)} | "
                  f"ph1 {diff_regions(ctx, 1, ctx.advice(1), a1)}", flush=True)
