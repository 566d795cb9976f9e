"""The standalone BabyBear NTT (plk_ntt_dev): forward DIF natural -> bit-reversed against an
O(n^2) DFT at small sizes, forward/inverse round trip and linearity at 2^20-2^23."""
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


@pytest.mark.parametrize("k", [16, 20, 23])
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
