#!/usr/bin/env python3
"""Config 2 (verify_mul_witness 256^2 P=32, graph replay): where the host time
of a call goes, and whether two contexts alternating (two independent stream
sets, so call j + 1 runs beside call j) beat one.

    python tools/probes/vmhost.py
"""
import ctypes as ct
import json
import os
import sys
import time
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
import halo2_svd041_amd as hs
from halo2_svd041_amd import zk
from halo2_svd041_amd._lib import lib
from bench import gen_matmul_input, gamma_for

N = int(os.environ.get("VM_N", "256"))
P = 32
dev = torch.device("cuda", 0)
a, b = gen_matmul_input(N, N, N, 0)
ta, tb = (torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev) for x in (a, b))
gs = [gamma_for(k) for k in range(400)]
out = {}


def timed(fn, iters=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(iters):
        fn(k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / iters * 1e3, (t2 - t0) / iters * 1e3


ctxs = [hs.Context(device=0, precision_bits=P, lookup_bits=19) for _ in range(2)]
for c in ctxs:
    c.set_option("lanes", 1)
for c in ctxs:
    for k in range(6):
        hs.verify_mul_witness(c, ta, tb, gs[k])
    c.sync()
c0 = ctxs[0]
ce = hs.Context(device=0, precision_bits=P, lookup_bits=19)       # eager (no graph)
ce.set_option("graph", 0)
ce.set_option("lanes", 1)
cel = hs.Context(device=0, precision_bits=P, lookup_bits=19)      # eager, two lanes
cel.set_option("graph", 0)
cel.set_option("lanes", 2)
for c in (ce, cel):
    for k in range(6):
        hs.verify_mul_witness(c, ta, tb, gs[k])
    c.sync()
for rnd in range(3):
    for name, c in (("eager_one_ctx", ce), ("eager_lanes2", cel)):
        h, s = timed(lambda k: hs.verify_mul_witness(c, ta, tb, gs[k]))
        out.setdefault(name, []).append({"host_ms": round(h, 4), "step_ms": round(s, 4)})
cl = hs.Context(device=0, precision_bits=P, lookup_bits=19)
cl.set_option("lanes", 2)
for k in range(10):
    hs.verify_mul_witness(cl, ta, tb, gs[k])
cl.sync()
for rnd in range(3):
    h, s = timed(lambda k: hs.verify_mul_witness(cl, ta, tb, gs[k]))
    out.setdefault("lanes2", []).append({"host_ms": round(h, 4), "step_ms": round(s, 4)})
    h, s = timed(lambda k: hs.verify_mul_witness(c0, ta, tb, gs[k]))
    out.setdefault("one_ctx", []).append({"host_ms": round(h, 4), "step_ms": round(s, 4)})
    h, s = timed(lambda k: hs.verify_mul_witness(ctxs[k & 1], ta, tb, gs[k]))
    out.setdefault("two_ctx_alternating", []).append({"host_ms": round(h, 4), "step_ms": round(s, 4)})
# pieces of the host call
cnt = zk.Counts()
args = [zk._words_arg(g) for g in gs]
ap, bp = ta.data_ptr(), tb.data_ptr()
L = lib()
h, s = timed(lambda k: L.svdw_verify_mul_witness(c0.handle, ap, bp, N, N, N, 1, args[k], ct.byref(cnt)))
out["c_call_only"] = {"host_ms": round(h, 4), "step_ms": round(s, 4)}
raw = zk._torch_stream(c0)
h, s = timed(lambda k: L.svdw_stream_wait(c0.handle, raw))
out["stream_wait_only"] = {"host_ms": round(h, 4)}
h, s = timed(lambda k: zk._words_arg(gs[k]))
out["gamma_words_only"] = {"host_ms": round(h, 4)}
h, s = timed(lambda k: zk._torch_stream(c0))
out["torch_stream_lookup"] = {"host_ms": round(h, 4)}
out["graph_stats"] = [list(c.graph_stats()) for c in ctxs + [cl]]
print(json.dumps(out))
if os.environ.get("SVDW_HOST_TRACE"):
    sys.stderr.flush()
