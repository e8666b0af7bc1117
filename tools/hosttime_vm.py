#!/usr/bin/env python3
"""Host cost of one verify_mul_witness call (BASELINE config 2: 256^2, P=32),
enqueue only from a synced start, vs the pipelined step.

    python tools/hosttime_vm.py [--n 256] [--p 32]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import gamma_for, gen_matmul_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--p", type=int, default=32)
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    x, y = gen_matmul_input(a.n, a.n, a.n, 0)
    dx, dy = (torch.tensor(np.ascontiguousarray(t), dtype=torch.float64, device="cuda") for t in (x, y))
    ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    for i in range(5):
        hs.verify_mul_witness(ctx, dx, dy, gamma_for(i))
    ctx.sync()
    ts = []
    for i in range(20):
        ctx.sync()
        t0 = time.perf_counter()
        hs.verify_mul_witness(ctx, dx, dy, gamma_for(i))
        ts.append(time.perf_counter() - t0)
    ctx.sync()
    t0 = time.perf_counter()
    for i in range(50):
        hs.verify_mul_witness(ctx, dx, dy, gamma_for(i))
    t1 = time.perf_counter()
    ctx.sync()
    el = (time.perf_counter() - t0) / 50
    ts.sort()
    print(f"verify_mul {a.n}^2 P={a.p}: host call min {ts[0] * 1e3:.3f} med {ts[10] * 1e3:.3f} ms; "
          f"pipelined enqueue {(t1 - t0) / 50 * 1e3:.3f} ms/call, step {el * 1e3:.3f} ms")
    if os.environ.get("SVDW_HOST_TRACE"):
        ctx.sync()
        print("=== 3 pipelined calls", file=sys.stderr, flush=True)
        for i in range(3):
            hs.verify_mul_witness(ctx, dx, dy, gamma_for(i))
        ctx.sync()
    ctx.close()


if __name__ == "__main__":
    main()
