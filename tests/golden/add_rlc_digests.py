#!/usr/bin/env python3
"""Add the rlc_prefix phase-1 digests to the golden fixtures (tests/golden/svd_*.json).

With svdw_set_option("rlc_prefix", 1) the phase-1 stream starts with the two
ctx_gate constant cells that examples/svd_example.rs:183's
rlc.load_rlc_cache((ctx_gate, ctx_rlc), gate, 1) appends, as the Python oracle
restates it (oracle/pyoracle.py load_rlc_cache_1: recalled axiom-eth RlcChip,
parity unpinned). For every fixture entry this computes that stream with the
Python oracle on the fixture's stored inputs, checks that it is [1, 0] followed
by the fixture's own phase-1 stream (whose digest the C oracle reproduces), and
stores its SHA-256 and length as sha256_advice1_rlc / advice1_rlc; and the
RLC context's own cells [E(one), E(zero), W(gamma)] (digest and the phase-1
sources of its two copies) as rlc_trace.

    python tests/golden/add_rlc_digests.py
"""
import glob
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import pyoracle as po  # noqa: E402


def _f64(hexes, shape=None):
    a = np.array([struct.unpack("<d", struct.pack("<Q", int(h, 16)))[0] for h in hexes])
    return a.reshape(shape) if shape else a


def _cells(vals):
    return np.array([[(x >> (64 * i)) & ((1 << 64) - 1) for i in range(4)] for x in vals], dtype=np.uint64)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


for path in sorted(glob.glob(os.path.join(HERE, "svd_*.json"))):
    with open(path) as fh:
        case = json.load(fh)
    N, M, g = case["N"], case["M"], int(case["gamma"])
    for exp in case["expected"]:
        d = case["inputs"][exp["input"]]
        m, u, v, dd = (_f64(d["m"], (N, M)), _f64(d["u"], (N, N)), _f64(d["v"], (M, M)), _f64(d["d"]))
        p = exp["precision_bits"]
        w = po.svd_witness(m.tolist(), u.tolist(), v.tolist(), dd.tolist(), p, case["lookup_bits"], g,
                           rlc_prefix=True)
        a1 = _cells(w.ctx1.advice)
        assert w.ctx1.advice[:2] == [1, 0]
        assert _sha(a1[2:]) == exp["sha256_advice1"], (path, exp["input"], p)
        exp["advice1_rlc"] = int(a1.shape[0])
        exp["sha256_advice1_rlc"] = _sha(a1)
        # ctx_rlc itself: [E(one), E(zero), W(gamma)], E cells copying the two
        # ctx_gate constants at the head of phase 1 (depends on gamma only)
        r = _cells(w.rlc.advice)
        assert [(a.ctx is w.ctx1, a.idx, dst) for a, dst in w.rlc.copies] == [(True, 0, 0), (True, 1, 1)]
        case["rlc_trace"] = {"cells": int(r.shape[0]), "sha256": _sha(r),
                             "copies": [[1, 0], [1, 1]]}
    with open(path, "w") as fh:
        json.dump(case, fh, indent=1)
        fh.write("\n")
    print("updated", os.path.basename(path))
