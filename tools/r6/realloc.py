"""Round-6 diagnostic: is the per-process spread of the 1024^2 step (1.90 vs
2.02 ms on one box) a property of where the engine's buffers land? One process:
a context is created, warmed, timed (30 steps), closed, and created again --
with a differently sized torch allocation held in between -- several times."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import gen_input, step_gammas  # noqa: E402


def main():
    import torch
    import halo2_svd041_amd as hs
    dev = torch.device("cuda", 0)
    m, u, d, v = gen_input(1024, 1024, 0)
    inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    hold = []
    for r in range(int(os.environ.get('REALLOC_N', '6'))):
        ctx = hs.Context(device=0, precision_bits=63, lookup_bits=19)
        ptrs = []
        for g in step_gammas(0, 3, offset=10 ** 6):
            hs.svd_witness(ctx, *inp, g)
            ctx.sync()
            ptrs.append([hex(ctx.advice_device_ptr(0)), hex(ctx.lookup_device_ptr(0)),
                         hex(ctx.advice_device_ptr(1)), hex(ctx.lookup_device_ptr(1))])
        ctx.sync()
        res = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for g in step_gammas(0, 30):
                hs.svd_witness(ctx, *inp, g)
            ctx.sync()
            res.append(round((time.perf_counter() - t0) / 30 * 1e3, 4))
        # the same witness with the streams serialised: each kernel alone
        ctx.set_option("overlap", 0)
        ctx.set_option("phase1_overlap", 0)
        ctx.set_option("pipeline", 0)
        hs.svd_witness(ctx, *inp, 5)
        ctx.sync()
        ctx.profile(True, "")
        hs.svd_witness(ctx, *inp, 5)
        ctx.sync()
        prof = {x["name"]: round(x["total_ms"], 4) for x in ctx.profile_collect()}
        ctx.profile(False)
        top = dict(sorted(prof.items(), key=lambda kv: -kv[1])[:6])
        print(json.dumps({"alloc": r, "ms": res, "ptrs": ptrs[:2], "serial": top}), flush=True)
        ctx.close()
        hold.append(torch.empty((r + 1) * 37 * 2 ** 20 + 12345, dtype=torch.uint8, device=dev))


if __name__ == "__main__":
    main()
