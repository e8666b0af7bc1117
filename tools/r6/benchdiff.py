"""Round-6 diagnostic for VERDICT #4: bench.py's 512^2 line reads ~4.5 % above
tools/ab.py's median on the same box. One process, alternating loops that
differ in one thing each: fresh gamma per step (bench.py) or one gamma (ab.py),
and whether every option is set again before the loop (ab.py does)."""
import argparse
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench import gen_input, gamma_for, step_gammas  # noqa: E402
from ab import DEFAULTS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--p", type=int, default=32)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    N = M = a.n
    m, u, d, v = gen_input(N, M, 0)
    dev = torch.device("cuda", 0)
    inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    cells = sum(hs.plan_svd(N, M, a.p, 19)[k] for k in ("advice0", "advice1"))
    fresh = step_gammas(0, a.steps)
    fixed = [gamma_for(0)] * a.steps
    variants = {"fresh": (fresh, False), "fixed": (fixed, False), "fresh+opts": (fresh, True),
                "fixed+opts": (fixed, True)}
    for g in step_gammas(0, 3, offset=10 ** 6):
        hs.svd_witness(ctx, *inp, g)
    ctx.sync()
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for name, (gs, opts) in variants.items():
            if opts:
                for k, val in DEFAULTS.items():
                    ctx.set_option(k, val)
            hs.svd_witness(ctx, *inp, gs[0])
            ctx.sync()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for g in gs:
                hs.svd_witness(ctx, *inp, g)
            ctx.sync()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / a.steps * 1e3)
    for name, r in res.items():
        med = statistics.median(r)
        print(f"{name:12s} median {med:.4f} ms -> {cells / med / 1e6:.2f} G  (in order {' '.join(f'{x:.4f}' for x in r)})")


if __name__ == "__main__":
    main()
