"""Round-6: an option A/B across buffer placements. Each round holds a
differently sized torch allocation first (so the engine's cell streams land
elsewhere), then times a fresh context per variant (median of 3 x 30 steps).
VARIANTS="name:opt=v,opt=v;name2:..." (default stage_rot 0 / 1)."""
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
    n = int(os.environ.get("PA_N", "1024"))
    p = int(os.environ.get("PA_P", "63"))
    steps = int(os.environ.get("PA_STEPS", "30"))
    variants = []
    for spec in os.environ.get("VARIANTS", "rot0:stage_rot=0;rot1:stage_rot=1").split(";"):
        name, _, rest = spec.partition(":")
        variants.append((name, [(k, int(v)) for k, v in (kv.split("=") for kv in rest.split(",") if kv)]))
    dev = torch.device("cuda", 0)
    m, u, d, v = gen_input(n, n, 0)
    inp = tuple(torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    hold = []
    for r in range(int(os.environ.get("PA_ROUNDS", "5"))):
        row = {"round": r}
        for name, opts in variants:
            ctx = hs.Context(device=0, precision_bits=p, lookup_bits=19)
            for k, val in opts:
                ctx.set_option(k, val)
            for g in step_gammas(0, 3, offset=10 ** 6):
                hs.svd_witness(ctx, *inp, g)
            ctx.sync()
            res = []
            for rep in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for g in step_gammas(0, steps):
                    hs.svd_witness(ctx, *inp, g)
                ctx.sync()
                res.append((time.perf_counter() - t0) / steps * 1e3)
            row[name] = round(sorted(res)[1], 4)
            ctx.close()
        print(json.dumps(row), flush=True)
        hold.append(torch.empty((r + 1) * 37 * 2 ** 20 + 12345, dtype=torch.uint8, device=dev))


if __name__ == "__main__":
    main()
