"""Golden fixtures (tests/golden/*.json, made by tests/golden/make_golden.py from
the reference's own input-creator.py): inputs as f64 bit patterns, expected
SHA-256 digests of the witness streams, counts and constraint verdicts.

CPU: the C oracle reproduces every digest; the JSON-parse modes differ as the
fixture says. GPU: the HIP engine reproduces every digest.
"""
import glob
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import corc

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "svd_*.json")))


def _f64(hexes, shape=None):
    a = np.array([struct.unpack("<d", struct.pack("<Q", int(h, 16)))[0] for h in hexes])
    return a.reshape(shape) if shape else a


def _inputs(case, key):
    N, M = case["N"], case["M"]
    d = case["inputs"][key]
    return (_f64(d["m"], (N, M)), _f64(d["u"], (N, N)), _f64(d["v"], (M, M)), _f64(d["d"]))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def _load(path):
    with open(path) as fh:
        return json.load(fh)


def test_fixtures_present():
    assert len(FIXTURES) >= 6


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_c_oracle_matches_golden(path):
    case = _load(path)
    g = int(case["gamma"])
    for exp in case["expected"]:
        m, u, v, d = _inputs(case, exp["input"])
        a0, l0, a1 = corc.svd_witness(m, u, v, d, exp["precision_bits"], case["lookup_bits"], g)
        assert a0.shape[0] == exp["advice0"] and a1.shape[0] == exp["advice1"]
        assert l0.shape[0] == exp["lookup0"]
        assert _sha(a0) == exp["sha256_advice0"]
        assert _sha(l0) == exp["sha256_lookup0"]
        assert _sha(a1) == exp["sha256_advice1"]


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_golden_known_answers(path):
    """README.md:93 on the reference generator's files: matrix verifies at every P;
    matrix-wrong fails at P >= 42 and (reference weakness) passes at P = 32."""
    case = _load(path)
    for exp in case["expected"]:
        wrong = exp["input"].startswith("matrix-wrong")
        if not wrong:
            assert exp["constraints_satisfied"], exp
        elif exp["precision_bits"] >= 42:
            assert not exp["constraints_satisfied"], exp
        else:
            assert exp["constraints_satisfied"], exp


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_rlc_prefix_golden_consistent(path):
    """The rlc_prefix phase-1 digests (tests/golden/add_rlc_digests.py: the Python
    oracle's load_rlc_cache(.., 1) restatement, parity unpinned) are the two
    ctx_gate constants [1, 0] followed by the C oracle's phase-1 stream."""
    case = _load(path)
    g = int(case["gamma"])
    for exp in case["expected"]:
        m, u, v, d = _inputs(case, exp["input"])
        _, _, a1 = corc.svd_witness(m, u, v, d, exp["precision_bits"], case["lookup_bits"], g)
        head = np.array([[1, 0, 0, 0], [0, 0, 0, 0]], dtype=np.uint64)
        both = np.concatenate([head, a1])
        assert both.shape[0] == exp["advice1_rlc"]
        assert _sha(both) == exp["sha256_advice1_rlc"]


def test_serde_parse_mode_changes_p63_witness():
    """serde_json default parsing differs by 1 ulp on some values; at P=63 the
    quantized cells (hence the digests) differ, at P=32 they typically do not."""
    case = _load(os.path.join(HERE, "golden", "svd_8x8_s5.json"))
    assert case["inputs"]["matrix/serde"]["ulp_diffs_vs_correct"] > 0
    by = {(e["input"], e["precision_bits"]): e["sha256_advice0"] for e in case["expected"]}
    assert by[("matrix/correct", 63)] != by[("matrix/serde", 63)]


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_engine_matches_golden(gpu_ctx_factory, path):
    import halo2_svd041_amd as hs
    case = _load(path)
    g = int(case["gamma"])
    for exp in case["expected"]:
        m, u, v, d = _inputs(case, exp["input"])
        ctx = gpu_ctx_factory(exp["precision_bits"], case["lookup_bits"])
        hs.svd_witness(ctx, m, u, v, d, g)
        assert _sha(ctx.advice(0)) == exp["sha256_advice0"]
        assert _sha(ctx.lookups(0)) == exp["sha256_lookup0"]
        assert _sha(ctx.advice(1)) == exp["sha256_advice1"]


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_engine_rlc_prefix_golden(gpu_ctx_factory, path):
    """rlc_prefix on: the engine's phase-1 stream (with load_rlc_cache's two
    ctx_gate cells) matches the golden digest; phase 0 is unchanged."""
    import halo2_svd041_amd as hs
    case = _load(path)
    g = int(case["gamma"])
    for exp in case["expected"]:
        m, u, v, d = _inputs(case, exp["input"])
        ctx = gpu_ctx_factory(exp["precision_bits"], case["lookup_bits"])
        ctx.set_option("rlc_prefix", 1)
        hs.svd_witness(ctx, m, u, v, d, g)
        assert _sha(ctx.advice(0)) == exp["sha256_advice0"]
        assert _sha(ctx.advice(1)) == exp["sha256_advice1_rlc"]


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_engine_from_raw_input_files(gpu_ctx_factory, path):
    """End to end from the generator's raw data/matrix.in: native serde-default
    parse -> engine witness == the golden digests of the serde-parsed input."""
    import halo2_svd041_amd as hs
    case = _load(path)
    base = os.path.basename(path)[:-5]
    g = int(case["gamma"])
    for exp in case["expected"]:
        name, mode = exp["input"].split("/")
        if mode != "serde":
            continue
        arrs = hs.parse_svd_input(os.path.join(os.path.dirname(path), "inputs",
                                               f"{base}_{name}.in"), "serde")
        ctx = gpu_ctx_factory(exp["precision_bits"])
        hs.svd_witness(ctx, arrs["m"], arrs["u"], arrs["v"], arrs["d"], g)
        assert _sha(ctx.advice(0)) == exp["sha256_advice0"]
        assert _sha(ctx.lookups(0)) == exp["sha256_lookup0"]
        assert _sha(ctx.advice(1)) == exp["sha256_advice1"]


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_rlc_trace_golden(path):
    """svdw_rlc_trace (the ctx_rlc stream of load_rlc_cache(.., 1), recalled
    axiom-eth construction, parity unpinned): the engine's three RLC cells and
    their copy sources equal the golden rlc_trace the Python oracle produced
    (tests/golden/add_rlc_digests.py); a host-only planning context suffices,
    the trace is host data. Without rlc_prefix there is no trace."""
    import halo2_svd041_amd as hs
    case = _load(path)
    g = int(case["gamma"])
    exp = case["expected"][0]
    m, u, v, d = _inputs(case, exp["input"])
    ctx = hs.Context(device=-1, precision_bits=exp["precision_bits"], lookup_bits=case["lookup_bits"])
    hs.svd_witness(ctx, m, u, v, d, g)
    assert ctx.rlc_trace() is None
    ctx.set_option("rlc_prefix", 1)
    hs.svd_witness(ctx, m, u, v, d, g)
    tr = ctx.rlc_trace()
    want = case["rlc_trace"]
    assert tr["cells"].shape[0] == want["cells"]
    assert _sha(tr["cells"]) == want["sha256"]
    assert [list(c) for c in tr["copies"]] == want["copies"]
    ctx.close()
