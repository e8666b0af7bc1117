#!/usr/bin/env python3
"""Host cost of one svd_witness call (enqueue only, from a synced start) vs the
pipelined step time, at 512^2 P=32 and 1024^2 P=63. When the host call is as
long as the step, the step is host-bound (launch overhead), not GPU-bound.

    python tools/probes/hosttime.py
"""
import sys, time, os
WORLD = int(os.environ.get("HT_WORLD", "1"))   # >1: time rank 0 of a row-sharded witness
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import halo2_svd041_amd as hs
from bench import gen_input, gamma_for
for N in (512, 1024):
    m, u, d, v = gen_input(N, N, 0)
    dev = torch.device("cuda", 0)
    dm, du, dv, dd = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (m, u, v, d))
    ctx = hs.Context(device=0, precision_bits=32 if N == 512 else 63, lookup_bits=19)
    if WORLD > 1:
        ctx.set_shard(0, WORLD)
    for _ in range(3): hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(0))
    ctx.sync()
    ts = []
    for _ in range(10):
        ctx.sync()
        t0 = time.perf_counter(); hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(0)); t1 = time.perf_counter()
        ts.append(t1 - t0)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(20): hs.svd_witness(ctx, dm, du, dv, dd, gamma_for(0))
    t1 = time.perf_counter()
    ctx.sync(); el = (time.perf_counter() - t0) / 20
    print(N, "host call (after sync) ms: min %.3f med %.3f" % (min(ts) * 1e3, sorted(ts)[5] * 1e3),
          "pipelined: host enqueue %.3f ms/call, step ms %.3f" % ((t1 - t0) / 20 * 1e3, el * 1e3))
    ctx.close()
