#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the dev container).

Inputs come from the reference's own generator, /root/reference/input-creator.py
(run unmodified with runpy in a temporary working directory after seeding
numpy's global RNG, since the script itself is unseeded: input-creator.py:24,28,47-48).
It writes data/matrix.in and data/matrix-wrong.in as JSON (json.dump, Python
repr floats); both files are parsed two ways:
  * "correct": Python's correctly rounded float parsing, and
  * "serde": an emulation of serde_json 1.0's default (non float_roundtrip)
    path f64_from_parts: (significand as f64) then one * or / by 10^|exp|
    (serde_json is the reference's parser,
    examples/svd_example.rs:330, Cargo.toml:16).
Each fixture stores the inputs as f64 bit patterns (hex) and the expected
witness digests (SHA-256 of the canonical 32-byte LE cell streams + counts)
computed by the pure-Python oracle and cross-checked against the C oracle,
plus the constraint-checker verdict (README.md:93 known-answer behaviour).

    python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import runpy
import struct
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import corc  # noqa: E402
import pyoracle as po  # noqa: E402

CASES = [  # (N, M, seed)
    (4, 4, 1), (4, 3, 2), (3, 4, 3), (6, 6, 4), (8, 8, 5), (5, 7, 6),
]
PRECISIONS = [32, 42, 63]
LOOKUP_BITS = 19
POW10 = [float(f"1e{k}") for k in range(309)]


def serde_f64(s: str) -> float:
    """serde_json default f64 parse of one JSON number token."""
    neg = s.startswith("-")
    t = s[1:] if neg else s
    mant, _, exp = t.replace("E", "e").partition("e")
    ip, _, fp = mant.partition(".")
    digits = (ip + fp).lstrip("0") or "0"
    sig = int(ip + fp)
    if sig >= 1 << 64:
        raise ValueError("significand overflow path not emulated")
    e = (int(exp) if exp else 0) - len(fp)
    f = float(sig)                    # u64 as f64: round to nearest even
    while True:
        if abs(e) < len(POW10):
            f = f * POW10[e] if e >= 0 else f / POW10[-e]
            break
        if f == 0.0:
            break
        f /= 1e308
        e += 308
    del digits
    return -f if neg else f


def load(path: str, mode: str):
    with open(path) as fh:
        txt = fh.read()
    if mode == "correct":
        obj = json.loads(txt)
    else:
        obj = json.loads(txt, parse_float=serde_f64, parse_int=lambda s: float(int(s)))
    return {k: np.array(obj[k], dtype=np.float64) for k in ("m", "u", "d", "v")}


def bits_hex(a: np.ndarray) -> list:
    return [f"{struct.unpack('<Q', struct.pack('<d', float(x)))[0]:016x}" for x in a.ravel()]


def sha(arr: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(arr, dtype=np.uint64).tobytes()).hexdigest()


def gamma_for(seed: int) -> int:
    return int.from_bytes(hashlib.sha256(f"svdw-gamma-{seed}".encode()).digest(), "little") % po.P_MOD


def make_case(ref: str, N: int, M: int, seed: int) -> dict:
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        argv = sys.argv
        try:
            os.chdir(td)
            np.random.seed(seed)
            sys.argv = ["input-creator.py", str(N), str(M)]
            runpy.run_path(os.path.join(ref, "input-creator.py"), run_name="__main__")
        finally:
            os.chdir(cwd)
            sys.argv = argv
        files = {name: os.path.join(td, "data", f"{name}.in") for name in ("matrix", "matrix-wrong")}
        parsed = {(name, mode): load(p, mode) for name, p in files.items()
                  for mode in ("correct", "serde")}
    g = gamma_for(seed)
    out = {"N": N, "M": M, "seed": seed, "gamma": str(g), "lookup_bits": LOOKUP_BITS,
           "generator": "input-creator.py (reference, unmodified) after np.random.seed(seed)",
           "inputs": {}, "expected": []}
    for (name, mode), arrs in parsed.items():
        out["inputs"][f"{name}/{mode}"] = {k: bits_hex(v) for k, v in arrs.items()}
        n_diff = sum(int(np.sum(parsed[(name, "correct")][k] != arrs[k])) for k in arrs)
        out["inputs"][f"{name}/{mode}"]["ulp_diffs_vs_correct"] = n_diff
        for P in PRECISIONS:
            w = po.svd_witness(arrs["m"].tolist(), arrs["u"].tolist(), arrs["v"].tolist(),
                               arrs["d"].tolist(), P, LOOKUP_BITS, g)
            a0 = np.array([[(x >> (64 * i)) & (2 ** 64 - 1) for i in range(4)] for x in w.ctx0.advice],
                          dtype=np.uint64)
            l0 = np.array([[(x >> (64 * i)) & (2 ** 64 - 1) for i in range(4)] for x in w.ctx0.lookups],
                          dtype=np.uint64).reshape(-1, 4)
            a1 = np.array([[(x >> (64 * i)) & (2 ** 64 - 1) for i in range(4)] for x in w.ctx1.advice],
                          dtype=np.uint64)
            c0, cl0, c1 = corc.svd_witness(arrs["m"], arrs["u"], arrs["v"], arrs["d"], P,
                                           LOOKUP_BITS, g)
            assert np.array_equal(a0, c0) and np.array_equal(l0, cl0) and np.array_equal(a1, c1), \
                "C oracle and Python oracle disagree"
            viol0 = po.check_constraints(w.ctx0, LOOKUP_BITS)
            viol1 = po.check_constraints(w.ctx1, LOOKUP_BITS)
            out["expected"].append({
                "input": f"{name}/{mode}", "precision_bits": P,
                "advice0": len(w.ctx0.advice), "lookup0": len(w.ctx0.lookups),
                "advice1": len(w.ctx1.advice),
                "sha256_advice0": sha(a0), "sha256_lookup0": sha(l0), "sha256_advice1": sha(a1),
                "first_cells_advice0": [str(x) for x in w.ctx0.advice[:4]],
                "last_cell_advice1": str(w.ctx1.advice[-1]),
                "constraints_satisfied": not viol0 and not viol1,
                "n_violations": len(viol0) + len(viol1),
                "err_svd": w.err_svd.hex(), "err_u": w.err_u.hex(),
            })
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    for N, M, seed in CASES:
        case = make_case(a.reference, N, M, seed)
        path = os.path.join(HERE, f"svd_{N}x{M}_s{seed}.json")
        with open(path, "w") as fh:
            json.dump(case, fh, indent=1)
        sat = {(e["input"], e["precision_bits"]): e["constraints_satisfied"] for e in case["expected"]}
        print(path, {k: v for k, v in sat.items()})


if __name__ == "__main__":
    main()
