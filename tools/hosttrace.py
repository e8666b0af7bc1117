#!/usr/bin/env python3
"""Host enqueue trace of pipelined svd_witness calls (SVDW_HOST_TRACE=1 markers
on stderr), for 1024^2 P=63 unsharded, rank 0 of 8, and 512^2 P=32.

    SVDW_HOST_TRACE=1 python tools/hosttrace.py 2> trace.txt
"""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import halo2_svd041_amd as hs  # noqa: E402
from bench import gamma_for, gen_input  # noqa: E402

for N, P, W in ((1024, 63, 1), (1024, 63, 8), (512, 32, 1)):
    m, u, d, v = gen_input(N, N, 0)
    dev = torch.device("cuda", 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)
                      for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=P, lookup_bits=19)
    if W > 1:
        ctx.set_shard(0, W)
    for _ in range(4):
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(0))
    ctx.sync()
    print(f"=== N={N} P={P} world={W}: 4 pipelined calls follow", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for k in range(4):
        print(f"--- call {k} at {(time.perf_counter() - t0) * 1e6:.1f} us", file=sys.stderr, flush=True)
        hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(k))
    ctx.sync()
    print(f"--- synced at {(time.perf_counter() - t0) * 1e6:.1f} us", file=sys.stderr, flush=True)
    ctx.close()
