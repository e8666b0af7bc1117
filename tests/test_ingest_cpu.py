"""Native input parser (svdw_parse_svd_input) against the
golden fixtures: the raw data/matrix.in files written by the reference's
input-creator.py parse to exactly the f64 bits stored in the golden JSON, in
both the serde_json-default and the correctly rounded mode."""
import glob
import json
import os
import struct

import numpy as np
import pytest

import halo2_svd041_amd as hs

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INPUTS = sorted(glob.glob(os.path.join(GOLD, "inputs", "*.in")))


def _bits(a):
    return [f"{struct.unpack('<Q', struct.pack('<d', float(x)))[0]:016x}" for x in np.ravel(a)]


def _f(tok, mode):
    text = '{"m": [[%s]], "u": [[1]], "v": [[1]], "d": [1]}' % tok
    return hs.parse_svd_input(text, mode)["m"][0, 0]


def test_fixture_inputs_present():
    assert len(INPUTS) == 12


@pytest.mark.parametrize("path", INPUTS, ids=os.path.basename)
@pytest.mark.parametrize("mode", ["serde", "correct"])
def test_parse_matches_golden_bits(path, mode):
    base = os.path.basename(path)[:-3]                     # svd_4x4_s1_matrix(-wrong)
    case, name = base.rsplit("_matrix", 1)
    name = "matrix" + name
    with open(os.path.join(GOLD, case + ".json")) as fh:
        want = json.load(fh)["inputs"][f"{name}/{mode}"]
    got = hs.parse_svd_input(path, mode)
    N, M = got["m"].shape
    assert got["u"].shape == (N, N) and got["v"].shape == (M, M) and got["d"].shape == (min(N, M),)
    for k in ("m", "u", "d", "v"):
        assert _bits(got[k]) == want[k], k


def test_serde_mode_differs_from_correct_rounding_somewhere():
    diffs = 0
    for path in INPUTS:
        a, b = hs.parse_svd_input(path, "serde"), hs.parse_svd_input(path, "correct")
        diffs += sum(int(np.sum(a[k] != b[k])) for k in a)
    assert diffs > 0          # ~10 % of input-creator values


@pytest.mark.parametrize("tok", ["0", "-0.0", "1", "-17", "0.1", "1e-05", "2.5e3", "123456789012345678",
                                 "9.87654321e-300", "1.7976931348623157e308", "4.9e-324"])
def test_number_tokens(tok):
    got_c = _f(tok, "correct")
    assert _bits([got_c]) == _bits([float(tok)])
    got_s = _f(tok, "serde")
    # serde default: u64 significand then one * or / by 10^|e|, 1e308 steps below
    mant, _, exp = tok.lstrip("-").partition("e")
    ip, _, fp = mant.partition(".")
    sig, e = int(ip + fp), (int(exp) if exp else 0) - len(fp)
    f = float(sig)
    while True:
        if abs(e) <= 308:
            f = f * float(f"1e{e}") if e >= 0 else f / float(f"1e{-e}")
            break
        if f == 0.0:
            break
        f /= 1e308
        e += 308
    f = -f if tok.startswith("-") else f
    assert _bits([got_s]) == _bits([f])


@pytest.mark.parametrize("text", [
    '{"m": [[1, 2], [3]], "u": [[1]], "v": [[1]], "d": [1]}',        # ragged
    '{"m": [[1]], "u": [[1]], "v": [[1]]}',                           # missing d
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1]} x',               # trailing
    '{"m": [[1.]], "u": [[1]], "v": [[1]], "d": [1]}',                # bad number
    '{"m": [[123456789012345678901234]], "u": [[1]], "v": [[1]], "d": [1]}',  # > u64
])
def test_malformed_inputs_rejected(text):
    with pytest.raises(hs.SvdwError):
        hs.parse_svd_input(text, "serde")


def test_unknown_keys_skipped_and_key_order_free():
    text = '{"note": {"a": [1, "x"]}, "d": [2.5], "v": [[1.0]], "u": [[-1e0]], "m": [[0.5]]}'
    got = hs.parse_svd_input(text, "serde")
    assert got["m"][0, 0] == 0.5 and got["u"][0, 0] == -1.0 and got["d"][0] == 2.5
