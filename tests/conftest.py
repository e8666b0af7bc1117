import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

P_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def gen_svd_input(N, M, seed):
    """input-creator.py:23-30 recipe with a seeded RandomState (same call order)."""
    rs = np.random.RandomState(seed)
    m = rs.uniform(-10, 10, size=(N, M))
    m = m / np.linalg.norm(m, ord=2) * rs.uniform(1, 100)
    U, D, V = np.linalg.svd(m)
    return m, U, D, V


def gamma_for(seed) -> int:
    """Fixed Fiat-Shamir stand-in: SHA-256("svdw-gamma-<seed>") mod p."""
    return int.from_bytes(hashlib.sha256(f"svdw-gamma-{seed}".encode()).digest(), "little") % P_MOD


def have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx_factory():
    if not have_gpu():
        pytest.skip("no HIP device")
    import halo2_svd041_amd as hs
    hs.zk.lib()  # raises loudly if libsvdw.so is missing
    ctxs = []

    def make(p, lb=19):
        c = hs.Context(device=0, precision_bits=p, lookup_bits=lb)
        ctxs.append(c)
        return c
    yield make
    for c in ctxs:
        c.close()
