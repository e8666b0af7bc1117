"""Round-6 diagnostic: per allocation (as realloc.py), the pipelined 1024^2
step beside plain torch passes over the phase-0 advice stream the step writes:
fill_ (memset-like), and a copy of its first half into its second. Does the
memory itself run slower in the slow placements, or only the witness's
pattern?"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import gen_input, step_gammas  # noqa: E402


def tb_s(f, nbytes, reps=5):
    import torch
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return round(nbytes * reps / (time.perf_counter() - t0) / 1e12, 3)


def main():
    import torch
    import halo2_svd041_amd as hs
    from halo2_svd041_amd import collect
    dev = torch.device("cuda", 0)
    m, u, d, v = gen_input(1024, 1024, 0)
    inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    hold = []
    for r in range(int(os.environ.get("REALLOC_N", "6"))):
        ctx = hs.Context(device=0, precision_bits=63, lookup_bits=19)
        for g in step_gammas(0, 3, offset=10 ** 6):
            hs.svd_witness(ctx, *inp, g)
        ctx.sync()
        res = []
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for g in step_gammas(0, 30):
                hs.svd_witness(ctx, *inp, g)
            ctx.sync()
            res.append(round((time.perf_counter() - t0) / 30 * 1e3, 4))
        adv = collect.stream_tensors(ctx, dev)[(0, 0)].view(-1)
        nb = adv.numel()
        half = nb // 2
        fill = tb_s(lambda: adv.fill_(7), nb)
        cp = tb_s(lambda: adv[half:2 * half].copy_(adv[:half]), 2 * half)
        print(json.dumps({"alloc": r, "ms": res, "fill_TBs": fill, "copy_TBs": cp, "GB": round(nb / 1e9, 2)}),
              flush=True)
        del adv
        ctx.close()
        hold.append(torch.empty((r + 1) * 37 * 2 ** 20 + 12345, dtype=torch.uint8, device=dev))


if __name__ == "__main__":
    main()
