"""The standalone NTTs -- BabyBear (plk_ntt_dev) and F29 (plk_ntt29_dev, the field of poly_mul
and the prover): forward DIF natural -> bit-reversed against an O(n^2) DFT at small sizes and an
independent numpy transform, forward/inverse round trip and linearity up to the 2-adicity."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
P = 2013265921
R = (1 << 32) % P


def to_mont(x):
    return ((x.astype(object) * R) % P).astype(np.uint32)


def from_mont(x):
    rinv = pow(R, P - 2, P)
    return ((x.astype(object) * rinv) % P).astype(np.int64)


def bitrev(i, k):
    return int(format(i, "0%db" % k)[::-1], 2)


@pytest.mark.parametrize("k", [1, 2, 5, 8, 10, 12, 13, 14])
def test_forward_vs_dft(hip, k):
    import torch
    n = 1 << k
    rng = np.random.default_rng(k)
    x = rng.integers(0, P, n, dtype=np.int64)
    w = pow(31, (P - 1) >> k, P)        # the library's root of order 2^k (generator 31)
    d = torch.from_numpy(to_mont(x).view(np.int32)).cuda()
    hip.ntt_dev(d, k, False, torch.cuda.current_stream())
    torch.cuda.synchronize()
    y = from_mont(d.cpu().numpy().view(np.uint32))
    xs = [int(v) for v in x]
    for j in list(range(min(n, 8))) + [n - 1]:
        want = sum(xs[i] * pow(w, i * j, P) for i in range(n)) % P
        assert y[bitrev(j, k)] == want, (k, j)


@pytest.mark.parametrize("k", [16, 20, 23, 24, 25, 27])   # 24+: three-pass plans, up to the 2-adicity
def test_roundtrip_and_linearity(hip, k):
    import torch
    n = 1 << k
    g = torch.Generator(device="cuda").manual_seed(k)
    a = torch.randint(0, P, (n,), dtype=torch.int64, device="cuda", generator=g)
    b = torch.randint(0, P, (n,), dtype=torch.int64, device="cuda", generator=g)
    st = torch.cuda.current_stream()
    A = a.to(torch.int32).clone()
    B = b.to(torch.int32).clone()
    S = ((a + b) % P).to(torch.int32).clone()
    for t in (A, B, S):
        hip.ntt_dev(t, k, False, st)
    # linearity (Montgomery form is linear too)
    lhs = (A.to(torch.int64) & 0xFFFFFFFF) + (B.to(torch.int64) & 0xFFFFFFFF)
    assert torch.equal(lhs % P, S.to(torch.int64) & 0xFFFFFFFF)
    hip.ntt_dev(A, k, True, st)
    torch.cuda.synchronize()
    # inverse is unscaled: A = n * a
    got = (A.to(torch.int64) & 0xFFFFFFFF)
    assert torch.equal(got, (a * n) % P)


def ntt_dif_reference(x, k, P=P, gen=31):
    """Independent numpy DIF NTT over BabyBear (or F29: P29, generator 3), natural order in,
    bit-reversed out, on the raw stored u32 values -- the transform commutes with the
    Montgomery scaling, so this is exactly what the GPU must produce from the same stored words."""
    a = x.astype(np.uint64) % P
    n = 1 << k
    w = pow(gen, (P - 1) >> k, P)
    for s in range(k - 1, -1, -1):
        h = 1 << s
        ws_ = pow(w, 1 << (k - s - 1), P)
        tw = np.ones(h, dtype=np.uint64)
        m = 1
        while m < h:
            tw[m:2 * m] = tw[:m] * np.uint64(pow(ws_, m, P)) % np.uint64(P)
            m *= 2
        a = a.reshape(n // (2 * h), 2, h)
        u, v = a[:, 0, :], a[:, 1, :]
        top = (u + v) % np.uint64(P)
        bot = (u + np.uint64(P) - v) % np.uint64(P) * tw % np.uint64(P)
        a = np.stack([top, bot], axis=1).reshape(n)
    return a


@pytest.mark.parametrize("k", [13, 14, 15, 17, 19, 20, 21, 22, 23, 24])
def test_forward_vs_numpy_reference(hip, k):
    """Every pass plan of the wave-tile engine (remainder pass of 1..10 bits on top, 10-bit
    passes below) against an independent full transform."""
    import torch
    rng = np.random.default_rng(100 + k)
    x = rng.integers(0, P, 1 << k, dtype=np.int64)
    d = torch.from_numpy(x.astype(np.int32)).cuda()
    hip.ntt_dev(d, k, False, torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    want = ntt_dif_reference(x, k)
    assert np.array_equal(got, want), k
    # inverse (unscaled) brings back n * x
    hip.ntt_dev(d, k, True, torch.cuda.current_stream())
    torch.cuda.synchronize()
    back = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(back, (x.astype(np.uint64) * np.uint64(1 << k)) % np.uint64(P))


@pytest.mark.parametrize("k,batch", [(10, 3), (14, 9), (20, 8), (22, 3)])
def test_batch_matches_single(hip, k, batch):
    """plk_ntt_batch_dev (arrays sharing each pass's launch, <= 8 per launch) is bit-identical
    to plk_ntt_dev on every array, forward and inverse."""
    import torch
    st = torch.cuda.current_stream()
    g = torch.Generator(device="cpu").manual_seed(k * 100 + batch)
    x = torch.randint(0, P, (batch, 1 << k), generator=g, dtype=torch.int64).to(torch.int32).cuda()
    for inv in (False, True):
        one = x.clone()
        for b in range(batch):
            hip.ntt_dev(one[b], k, inv, st)
        many = x.clone()
        hip.ntt_batch_dev(many, k, batch, inv, st)
        torch.cuda.synchronize()
        assert torch.equal(one, many), (k, batch, inv)


# ---- F29 (plk_ntt29_dev): the field poly_mul and the device prover transform in ----------------
P29 = 7 * (1 << 26) + 1


@pytest.mark.parametrize("k", [13, 14, 17, 20, 21, 22, 23, 24, 25, 26])
def test_f29_forward_vs_numpy_reference(hip, k):
    """Every pass plan (2^12 tiles to 2^20, 2^13 tiles above, 3-pass plans from 2^24) against
    the independent transform; outputs fully reduced; the unscaled inverse brings back n x."""
    import torch
    rng = np.random.default_rng(200 + k)
    x = rng.integers(0, P29, 1 << k, dtype=np.int64)
    d = torch.from_numpy(x.astype(np.int32)).cuda()
    st = torch.cuda.current_stream()
    hip.ntt29_dev(d, k, False, st)
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    if k <= 23:
        assert np.array_equal(got, ntt_dif_reference(x, k, P29, 3)), k
    assert int(got.max()) < P29
    hip.ntt29_dev(d, k, True, st)
    torch.cuda.synchronize()
    back = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(back, (x.astype(np.uint64) * np.uint64(pow(2, k, P29))) % np.uint64(P29))


def test_f29_batch_and_range(hip):
    import torch
    st = torch.cuda.current_stream()
    k, batch = 20, 9
    g = torch.Generator(device="cpu").manual_seed(29)
    x = torch.randint(0, P29, (batch, 1 << k), generator=g, dtype=torch.int64).to(torch.int32).cuda()
    for inv in (False, True):
        one = x.clone()
        for b in range(batch):
            hip.ntt29_dev(one[b], k, inv, st)
        many = x.clone()
        hip.ntt29_batch_dev(many, k, batch, inv, st)
        torch.cuda.synchronize()
        assert torch.equal(one, many), inv
    for bad in (12, 27):
        with pytest.raises(hip.PlonkHipError):
            hip.ntt29_dev(x[0], bad, False, st)


@pytest.mark.parametrize("field", ["bb", "f29"])
@pytest.mark.parametrize("k", [13, 17, 20, 21, 22, 24])
@pytest.mark.parametrize("pattern", ["max", "alt"])
def test_extreme_values_every_plan(hip, field, k, pattern):
    """Inputs at the top of the field (every word p - 1) and alternating 0 / p - 1: the lazy F29
    bounds (values < 4p forward, < 8p inverse, the multiply-free stage 0 of both directions, the
    {w, p - w} pair butterflies) at their largest, on every pass plan; forward against the numpy
    reference (k <= 23), inverse back to n x."""
    import torch
    p, gen = (P, 31) if field == "bb" else (P29, 3)
    fwd = hip.ntt_dev if field == "bb" else hip.ntt29_dev
    n = 1 << k
    x = np.full(n, p - 1, np.int64)
    if pattern == "alt":
        x[::2] = 0
    d = torch.from_numpy(x.astype(np.uint32).view(np.int32)).cuda()
    st = torch.cuda.current_stream()
    fwd(d, k, False, st)
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert int(got.max()) < p
    if k <= 23:
        assert np.array_equal(got, ntt_dif_reference(x, k, p, gen)), (field, k, pattern)
    fwd(d, k, True, st)
    torch.cuda.synchronize()
    back = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(back, (x.astype(np.uint64) * np.uint64(pow(2, k, p))) % np.uint64(p)), (field, k, pattern)


_TILE12_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = sys.argv[1:5]
import plonkhip as hip
import gen
from pyoracle import Oracle
from test_ntt_gpu import P, P29, ntt_dif_reference
hip.set_option("NTT_T13_MIN_K", 24)   # shapes the column tables: before plk_init
hip.init(0)
st = torch.cuda.current_stream()
for k in (21, 22):
    for p, g, fn in ((P29, 3, hip.ntt29_dev), (P, 31, hip.ntt_dev)):
        x = np.random.default_rng(k).integers(0, p, 1 << k, dtype=np.int64)
        d = torch.from_numpy(x.astype(np.int32)).cuda()
        fn(d, k, False, st)
        torch.cuda.synchronize()
        got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
        print("ntt", k, p, bool(np.array_equal(got, ntt_dif_reference(x, k, p, g))))
a, b = gen.poly_inputs(21, (1 << 20) - 3, (1 << 20) + 2)
print("poly_mul", hip.poly_mul(a, b) == Oracle().poly_mul_ntt(a, b))
"""


def test_tile12_three_pass_plans():
    """2^21 and 2^22 transforms on 2^12 tiles (PLK_OPT_NTT_T13_MIN_K = 24, set before plk_init: a
    child process): three-pass plans whose top pass is not the column tables' single high pass, so
    it multiplies lo * hi factors instead (round 5: with the table it gave wrong transforms) --
    forward against the numpy reference in both fields, and a 2^21 product against the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = [os.path.join(root, d) for d in ("plonk.c_amd", "oracle", "tests", os.path.join("tests", "golden"))]
    r = subprocess.run([sys.executable, "-c", _TILE12_SCRIPT] + paths, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith(("ntt", "poly_mul"))]
    assert len(lines) == 5 and all(ln.endswith("True") for ln in lines), r.stdout
