#!/usr/bin/env python3
"""Config 2: the caller-stream hand-off. lanes 1 / 2; torch's current stream the
default stream or a side stream; the hand-off as its own call
(svdw_stream_wait, "old") or inside svdw_verify_mul_witness_on ("on").
300 calls each, interleaved.

    python tools/probes/vmstream.py
"""
import json
import os
import sys
import time
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
import halo2_svd041_amd as hs
from bench import gen_matmul_input, gamma_for

N, P = 256, 32
dev = torch.device("cuda", 0)
a, b = gen_matmul_input(N, N, N, 0)
ta, tb = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (a, b))
gs = [gamma_for(k) for k in range(300)]
side = torch.cuda.Stream()
out = {}
ctxs = {}
for lanes in (1, 2):
    c = hs.Context(device=0, precision_bits=P, lookup_bits=19)
    c.set_option("lanes", lanes)
    for k in range(10):
        hs.verify_mul_witness(c, ta, tb, gs[k])
    with torch.cuda.stream(side):
        for k in range(10):
            hs.verify_mul_witness(c, ta, tb, gs[k])
    c.sync()
    ctxs[lanes] = c
torch.cuda.synchronize()
import ctypes as ct
from halo2_svd041_amd import zk
from halo2_svd041_amd._lib import lib


def old_call(c, g):
    cnt = zk.Counts()
    zk._after_torch(c)
    zk.check(lib().svdw_verify_mul_witness(c.handle, ta.data_ptr(), tb.data_ptr(), N, N, N, 1,
                                           zk._words_arg(g), ct.byref(cnt)))


for rnd in range(3):
    for lanes in (1, 2):
        c = ctxs[lanes]
        torch.cuda.synchronize()
        c.sync()
        t0 = time.perf_counter()
        for k in range(300):
            old_call(c, gs[k])
        t1 = time.perf_counter()
        c.sync()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out.setdefault(f"lanes{lanes}_default_old", []).append(
            {"host_ms": round((t1 - t0) / 300 * 1e3, 4), "step_ms": round((t2 - t0) / 300 * 1e3, 4)})
        for sname in ("default", "side"):
            torch.cuda.synchronize()
            c.sync()
            if sname == "side":
                ctxm = torch.cuda.stream(side)
            else:
                ctxm = torch.cuda.stream(torch.cuda.default_stream())
            with ctxm:
                t0 = time.perf_counter()
                for k in range(300):
                    hs.verify_mul_witness(c, ta, tb, gs[k])
                t1 = time.perf_counter()
                c.sync()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
            out.setdefault(f"lanes{lanes}_{sname}", []).append(
                {"host_ms": round((t1 - t0) / 300 * 1e3, 4), "step_ms": round((t2 - t0) / 300 * 1e3, 4)})
print(json.dumps(out))
