"""Round-6 diagnostic: the 1024^2 step against the cell streams' placement
modulo 8 MiB ("cell_phase" -1: as hipMalloc puts them, 0..7: that MiB of the
period). One process; each round holds a differently sized torch allocation
first, so hipMalloc's own placement moves, then times a fresh context per
phase (3 x 30 steps)."""
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
    n = int(os.environ.get("PHASE_N", "1024"))
    p = int(os.environ.get("PHASE_P", "63"))
    phases = [int(x) for x in os.environ.get("PHASES", "-1,0,2,4,6").split(",")]
    dev = torch.device("cuda", 0)
    m, u, d, v = gen_input(n, n, 0)
    inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    hold = []
    for r in range(int(os.environ.get("PHASE_ROUNDS", "4"))):
        row = {"round": r}
        for ph in phases:
            ctx = hs.Context(device=0, precision_bits=p, lookup_bits=19)
            ctx.set_option("cell_phase", ph)
            for g in step_gammas(0, 3, offset=10 ** 6):
                hs.svd_witness(ctx, *inp, g)
            ctx.sync()
            res = []
            for rep in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for g in step_gammas(0, 30):
                    hs.svd_witness(ctx, *inp, g)
                ctx.sync()
                res.append((time.perf_counter() - t0) / 30 * 1e3)
            row[str(ph)] = round(sorted(res)[1], 4)
            row["adv0_" + str(ph)] = hex(ctx.advice_device_ptr(0))
            ctx.close()
        print(json.dumps(row), flush=True)
        hold.append(torch.empty((r + 1) * 37 * 2 ** 20 + 12345, dtype=torch.uint8, device=dev))


if __name__ == "__main__":
    main()
