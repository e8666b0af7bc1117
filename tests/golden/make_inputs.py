#!/usr/bin/env python3
"""Raw input files of the golden cases: data/matrix.in and data/matrix-wrong.in
exactly as the reference's input-creator.py writes them (run unmodified, in a
temporary directory, after np.random.seed(seed) -- the recipe of make_golden.py),
saved as tests/golden/inputs/svd_<N>x<M>_s<seed>_<name>.in. They are data (the
generator's output), used to pin the native input parser
(svdw_parse_svd_input) against the parsed bits stored in the golden JSON.

    python tests/golden/make_inputs.py [--reference /root/reference]
"""
import argparse
import json
import os
import runpy
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import CASES, bits_hex, load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    out_dir = os.path.join(HERE, "inputs")
    os.makedirs(out_dir, exist_ok=True)
    for N, M, seed in CASES:
        with tempfile.TemporaryDirectory() as td:
            cwd, argv = os.getcwd(), sys.argv
            try:
                os.chdir(td)
                np.random.seed(seed)
                sys.argv = ["input-creator.py", str(N), str(M)]
                runpy.run_path(os.path.join(a.reference, "input-creator.py"), run_name="__main__")
            finally:
                os.chdir(cwd)
                sys.argv = argv
            with open(os.path.join(HERE, f"svd_{N}x{M}_s{seed}.json")) as fh:
                golden = json.load(fh)
            for name in ("matrix", "matrix-wrong"):
                src = os.path.join(td, "data", f"{name}.in")
                for mode in ("correct", "serde"):   # same bits as the golden fixture
                    arrs = load(src, mode)
                    want = golden["inputs"][f"{name}/{mode}"]
                    assert all(bits_hex(arrs[k]) == want[k] for k in ("m", "u", "d", "v")), \
                        (N, M, seed, name, mode)
                dst = os.path.join(out_dir, f"svd_{N}x{M}_s{seed}_{name}.in")
                shutil.copyfile(src, dst)
                print(dst)


if __name__ == "__main__":
    main()
