"""Device ingest (svdw_parse_svd_input_device, serde mode) against the host
parser (svdw_parse_svd_input, itself pinned on the reference generator's raw
files in tests/golden/inputs): the same values bit for bit on every accepted
input, and the same rejections on malformed text; then raw file -> device
parse -> witness -> golden digests, and the full BASELINE size."""
import glob
import json
import os
import time

import numpy as np
import pytest

import halo2_svd041_amd as hs

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _bits(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64)).view(np.uint64)


def _same(host, dev):
    for k in ("m", "u", "v", "d"):
        got = dev[k].cpu().numpy()
        assert got.shape == host[k].shape, k
        assert np.array_equal(_bits(got), _bits(host[k])), k


@pytest.fixture(scope="module")
def ctx():
    from conftest import have_gpu
    if not have_gpu():                   # (torch initialises the runtime first)
        pytest.skip("no HIP device")
    with hs.Context(device=0, precision_bits=63, lookup_bits=19) as c:
        yield c


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "inputs", "*.in"))))
def test_golden_files_match_host(ctx, path):
    _same(hs.parse_svd_input(path, "serde"), hs.parse_svd_input_device(ctx, path))


ACCEPTED = [
    '{"m": [[1, 2], [3, 4]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"note": {"a": [1, "x"]}, "d": [2.5], "v": [[1.0]], "u": [[-1e0]], "m": [[0.5]]}',
    '{"m":[[0,-0.0,1e-05,2.5E3,123456789012345678]],"u":[[9.87654321e-300]],'
    '"v":[[1.7976931348623157e308]],"d":[4.9e-324, 1e-400, 0e999]}',
    '{"x\\"y": [[1, [2, "]"]]], "flag": true, "n": null, "s": "a,b]", "m": [[7]], "u": [[1]],'
    ' "v": [[1]], "d": []}',
    '\n\t {"m" : [ [ 1 , 2 ] ] , "u":[[1]],"v":[[1]],"d":[1]}  \n',
    '{"m": [[], []], "u": [[1]], "v": [[1]], "d": [1]}',
]


@pytest.mark.parametrize("text", ACCEPTED)
def test_accepted_inputs_match_host(ctx, text):
    _same(hs.parse_svd_input(text, "serde"), hs.parse_svd_input_device(ctx, text))


REJECTED = [
    '{"m": [[1, 2], [3]], "u": [[1]], "v": [[1]], "d": [1]}',        # ragged
    '{"m": [[1]], "u": [[1]], "v": [[1]]}',                           # missing d
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1]} x',               # trailing
    '{"m": [[1.]], "u": [[1]], "v": [[1]], "d": [1]}',                # bad number
    '{"m": [[123456789012345678901234]], "u": [[1]], "v": [[1]], "d": [1]}',  # > u64
    '{"m": [[1,,2]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1,2,]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1],[2],], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1][2]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1 2]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1], 2], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [1, 2], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [[1]]}',
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1], "m": [[2]]}',
    '{"m": [[1]] "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [["1"]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[+1]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1e]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1e400000]}',
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1]',
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1]}}',
    '{"m" [[1]], "u": [[1]], "v": [[1]], "d": [1]}',
    '{"m": [[1]], "u": [[1]], "v": [[1]], "d": [1], "s": "x}',
]


@pytest.mark.parametrize("text", REJECTED)
def test_rejected_inputs_match_host(ctx, text):
    with pytest.raises(hs.SvdwError):
        hs.parse_svd_input(text, "serde")
    with pytest.raises(hs.SvdwError):
        hs.parse_svd_input_device(ctx, text)


def test_raw_file_to_witness_on_device(ctx):
    """input-creator.py's own file -> device parse -> witness, equal to the host
    parse -> witness (whose digests test_golden.py pins)."""
    path = os.path.join(GOLD, "inputs", "svd_6x6_s4_matrix.in")
    g = 123456789
    with hs.Context(device=0, precision_bits=63, lookup_bits=19) as c:
        dev = hs.parse_svd_input_device(c, path)
        hs.svd_witness(c, dev["m"], dev["u"], dev["v"], dev["d"], g)
        a0, a1, l0 = c.advice(0), c.advice(1), c.lookups(0)
    host = hs.parse_svd_input(path, "serde")
    with hs.Context(device=0, precision_bits=63, lookup_bits=19) as c:
        hs.svd_witness(c, host["m"], host["u"], host["v"], host["d"], g)
        assert np.array_equal(c.advice(0), a0) and np.array_equal(c.advice(1), a1)
        assert np.array_equal(c.lookups(0), l0)


def test_full_size_1024(ctx):
    """The BASELINE 1024 x 1024 witness input (json.dump(indent=4) of Python
    floats, as input-creator.py writes it: ~106 MB): device == host, bit for bit."""
    import torch
    from bench import gen_input
    m, u, d, v = gen_input(1024, 1024, 0)
    text = json.dumps({"m": m.tolist(), "u": u.tolist(), "d": d.tolist(), "v": v.tolist()},
                      indent=4).encode()
    t0 = time.perf_counter()
    host = hs.parse_svd_input(text, "serde")
    th = time.perf_counter() - t0
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to("cuda:0")
    hs.parse_svd_input_device(ctx, t)              # warm (scratch allocation)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev = hs.parse_svd_input_device(ctx, t)
    torch.cuda.synchronize()
    td = time.perf_counter() - t0
    _same(host, dev)
    print(f"\ningest 1024^2 ({len(text) / 1e6:.1f} MB): host parse {th * 1e3:.1f} ms, "
          f"device parse {td * 1e3:.2f} ms (text resident in HBM)")
