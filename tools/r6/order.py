"""Round-6 diagnostic: does the order in which the engine context and torch's
first device tensors are created change the pipelined step? (`first` = ctx:
bench.py's order, the context's three streams created before torch touches the
device; `first` = tensors: tools/ab.py's and shard_sim.py's order.) One process
per order; bench.py's loop otherwise (fresh gamma, 3 warm-up steps)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import gen_input, step_gammas  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", choices=["ctx", "tensors", "setdev"], required=True)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--p", type=int, default=63)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import torch
    import halo2_svd041_amd as hs
    m, u, d, v = gen_input(a.n, a.n, 0)
    dev = torch.device("cuda", 0)
    mk = lambda: tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa: E731
                       for x in (m, u, v, d))
    if a.first == "tensors":
        inp = mk()
        ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
    else:
        if a.first == "setdev":
            torch.cuda.set_device(0)
        ctx = hs.Context(device=0, precision_bits=a.p, lookup_bits=19)
        inp = mk()
    for g in step_gammas(0, 3, offset=10 ** 6):
        hs.svd_witness(ctx, *inp, g)
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for g in step_gammas(0, a.steps):
        hs.svd_witness(ctx, *inp, g)
    ctx.sync()
    torch.cuda.synchronize()
    print(json.dumps({"first": a.first, "n": a.n, "ms": round((time.perf_counter() - t0) / a.steps * 1e3, 4)}))


if __name__ == "__main__":
    main()
