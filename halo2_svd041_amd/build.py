"""Build libsvdw.so in-tree for gfx950 (hipcc; no JIT cache, travels with the repo).

    python -m halo2_svd041_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libsvdw.so")
SOURCES = ["kernels.hip", "ingest_dev.hip", "engine.cpp"]
HEADERS = ["fr.hpp", "prog.hpp", "kernels.hpp", "crt_tables.hpp", "ingest.hpp", "ingest_dev.hpp"]
ARCH = os.environ.get("SVDW_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "svdw.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-Wall", "-Wno-unused-function", "-o", OUT + ".tmp"]
    cmd += [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
