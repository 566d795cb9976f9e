"""GPU parity for poly_mul (reference src/poly.h:106-122 + trim src/poly.h:20-38) through
the C ABI: bit-exact coefficient bytes and trimmed length."""
import numpy as np
import pytest

import gen
from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_golden_cases(hip):
    g = load_golden("poly_mul.json")
    for c in g["cases"]:
        a, b = bytes.fromhex(c["a"]), bytes.fromhex(c["b"])
        assert hip.poly_mul(a, b).hex() == c["out"], (len(a), len(b))


@pytest.mark.parametrize("idx", range(9))
def test_golden_large_digests(hip, idx):
    c = load_golden("poly_mul.json")["large"][idx]
    a, b = gen.poly_inputs(c["seed"], c["la"], c["lb"])
    out = hip.poly_mul(a, b)
    assert len(out) == c["len"]
    assert gen.digest(np.frombuffer(out, np.uint8)) == c["sha256"]


@pytest.mark.parametrize("idx", range(3))
def test_golden_c3_size_digests(hip, idx):
    """Config C3 at its own size: reference digests of 2^18 x 2^18, 2^19 x 2^19 (the
    2^20-coefficient product) and a ragged shape around it (tests/golden/poly_mul_big.json,
    recorded from oracle/_ref by make_golden.py poly_big)."""
    c = load_golden("poly_mul_big.json")["large"][idx]
    a, b = gen.poly_inputs(c["seed"], c["la"], c["lb"])
    out = hip.poly_mul(a, b)
    assert len(out) == c["len"]
    assert gen.digest(np.frombuffer(out, np.uint8)) == c["sha256"]


def test_survey_digests(hip, oracle):
    for c in load_golden("poly_mul.json")["survey_xorshift"]:
        a, b = oracle.gen_survey_poly(c["n"])
        out = hip.poly_mul(a, b)
        assert len(out) == c["len"]
        assert "%08x" % oracle.digest31(np.frombuffer(out, np.uint8)) == c["digest31"]


# shapes straddling every dispatch boundary: direct (min <= 32), one workgroup (N <= 2^12),
# two passes (2^13..2^22), three passes (2^23+)
SHAPES = [(1, 1), (33, 33), (32, 1000), (33, 1000), (2048, 2049), (2049, 2048), (4097, 4),
          (4097, 33), (3000, 5000), (1 << 12, 1 << 12), ((1 << 13) + 1, 999),
          (1 << 15, (1 << 15) + 1), (100000, 3), (70000, 90000), ((1 << 19), (1 << 19)),
          ((1 << 20) + 3, (1 << 20) + 5), (3 * (1 << 20) + 4, (1 << 20) + 3),
          # wrapped products: la + lb - 1 = 2^K + e, e <= 16 (cyclic 2^K transform, the top e
          # coefficients computed directly)
          (4097, 4100), (8193, 8196), (8196, 8193), (8200, 8201), (8200, 8202), (16386, 100),
          ((1 << 16) + 2, (1 << 16)), (3 * (1 << 14) + 4, (1 << 14) + 3)]
# 2^24-point transforms (three-pass plans): F29 (min * 128 < p) and BabyBear (min above the F29
# bound, below the oracle's 998244353 one)
SHAPES += [(5000000, 3600000), (5000000, 3800000)]
# every wrap width e = 1..16 against the shortest transform-path operand (33 coefficients), both orders
SHAPES += [((1 << 13) - 32 + e, 33)[::1 if e % 2 else -1] for e in range(1, 17)]


@pytest.mark.parametrize("la,lb", SHAPES)
def test_shapes_vs_oracle(hip, oracle, la, lb):
    a, b = gen.poly_inputs(la * 31 + lb, la, lb)
    want = oracle.poly_mul(a, b) if la * lb <= (1 << 24) else oracle.poly_mul_ntt(a, b)
    ok = hip.poly_mul(a, b) == want   # (a failing assert on megabyte operands makes pytest diff them for minutes)
    assert ok, (la, lb)


def test_random_shapes_and_bytes_vs_oracle(hip, oracle):
    """80 seeded shapes drawn log-uniformly from 1 to 2^20 coefficients per operand (every dispatch
    path and transform size up to 2^21 points, wrapped or not), each with operands of one of four byte
    kinds -- canonical residues, any byte value, trailing zeros (an untrimmed input), sparse -- against
    the oracle's independent NTT over 998244353; the same products again as one batched launch
    (plk_poly_mul_batch_dev: one launch per pass for the whole batch of a transform size)"""
    rng = np.random.default_rng(0x600D)
    cases = []
    for t in range(80):
        la, lb = (int(2 ** rng.uniform(0, 20)) for _ in range(2))
        kind = t % 4
        a = rng.integers(0, 256 if kind == 1 else 17, la).astype(np.uint8)
        b = rng.integers(0, 256 if kind == 1 else 17, lb).astype(np.uint8)
        if kind == 2 and la > 1:
            a[-min(la - 1, 5):] = 0
        if kind == 3:
            a[rng.random(la) < 0.9] = 0
            b[rng.random(lb) < 0.9] = 0
        want = oracle.poly_mul_ntt(a, b)
        got = hip.poly_mul(a, b)
        assert got == want, (t, la, lb, kind)   # (bytes compare: no megabyte diff on failure)
        cases.append((a, b, want))
    # the products of at least 64 x 64 coefficients (the NTT paths) as ONE batch: it groups its jobs
    # by transform size, one launch per pass per size
    big = [(a, b, w) for a, b, w in cases if len(a) >= 64 and len(b) >= 64]
    pool = [x for a, b, _ in big for x in (a, b)]
    outs = _run_batch(hip, pool, [(2 * i, 2 * i + 1, 0) for i in range(len(big))])
    for (a, b, w), o in zip(big, outs):
        assert _trim(o) == w, (len(a), len(b))


def test_trailing_cancellation_and_zero(hip, oracle):
    # products whose top coefficients vanish: trimmed length < la + lb - 1
    a = np.zeros(5000, np.uint8); a[0] = 1; a[4000] = 0   # untrimmed input a = 1
    b = np.zeros(6000, np.uint8); b[10] = 3
    assert hip.poly_mul(a, b) == oracle.poly_mul(a, b)
    z = np.zeros(7000, np.uint8)
    assert hip.poly_mul(z, z) == bytes([0])
    # non-canonical coefficient bytes are reduced like hf_mul does
    a, b = gen.poly_inputs(5, 3000, 3000, modulus=256)
    assert hip.poly_mul(a, b) == oracle.poly_mul(a, b)


@pytest.mark.parametrize("la,lb", [(8193, 8196), (8200, 8202), ((1 << 13) - 32 + 7, 33), (70000, 90000)])
def test_trimmed_length_from_the_last_pass(hip, oracle, la, lb):
    """The transform path takes the trimmed length (src/poly.h:20-38) out of its last inverse
    pass: one store when the top coefficient a[la-1] b[lb-1] mod 17 is non-zero, else a block
    maximum per tile.  Leading bytes that are 0 mod 17 (17, 34, 0) force the second form, on
    wrapped shapes too (their top coefficients come from the direct fix-up)."""
    import torch
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    work = torch.zeros(max(hip.poly_mul_workspace(la, lb), 4), dtype=torch.uint8, device=dev)
    out = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
    nz = torch.full((4,), 0x7FFFFFFF, dtype=torch.int32, device=dev)   # stale value: must be replaced
    for ta, tb in [(None, None), (17, None), (None, 34), (0, 0), (17, 34)]:
        a, b = gen.poly_inputs(la + 7 * lb, la, lb)
        a, b = a.copy(), b.copy()
        if ta is not None:
            a[-1] = ta
            a[-3:-1] = [0, 17]          # the next coefficients vanish too
        if tb is not None:
            b[-1] = tb
        want = oracle.poly_mul(a, b) if la * lb <= (1 << 24) else oracle.poly_mul_ntt(a, b)
        assert hip.poly_mul(a, b) == want, (ta, tb)
        hip.poly_mul_dev(torch.from_numpy(a).to(dev), la, torch.from_numpy(b).to(dev), lb, out, nz, work, st)
        torch.cuda.synchronize()
        n = int(nz[0].item())
        assert (n or 1) == len(want), (ta, tb, n, len(want))
        assert bytes(out[:n or 1].cpu().numpy()) == want


def test_empty_operand_mirrors_reference(hip):
    assert hip.poly_mul(b"", b"\x03\x04") == bytes([0])


def test_device_api(hip, oracle):
    import torch
    dev = torch.device("cuda:0")
    la, lb = 300000, 200001
    a, b = gen.poly_inputs(8, la, lb)
    da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    out = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
    nz = torch.zeros(4, dtype=torch.int32, device=dev)
    work = torch.zeros(max(hip.poly_mul_workspace(la, lb), 4), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    for _ in range(2):
        hip.poly_mul_dev(da, la, db, lb, out, nz, work, st)
    torch.cuda.synchronize()
    n = int(nz[0].item()) or 1
    assert bytes(out[:n].cpu().numpy()) == oracle.poly_mul_ntt(a, b)


@pytest.mark.parametrize("m", [1835007, 1835008])
def test_all_sixteen_products(hip, m):
    """All coefficients 16 (the uncentered maximum: c_i = 256 min(i + 1, la, lb, la + lb - 1 - i),
    256 = 1 mod 17) at the old uncentered F29 boundary (min(la, lb) * 256 < p); both sides run
    over F29 now that coefficients enter centered (16 = -1)."""
    la, lb = m, m + 1000
    a = np.full(la, 16, np.uint8)
    b = np.full(lb, 16, np.uint8)
    i = np.arange(la + lb - 1, dtype=np.int64)
    want = (np.minimum(np.minimum(i + 1, la), np.minimum(lb, la + lb - 1 - i)) % 17).astype(np.uint8)
    nz = np.flatnonzero(want)
    want = want[:int(nz[-1]) + 1]
    assert hip.poly_mul(a, b) == want.tobytes()


@pytest.mark.parametrize("m", [3670016, 3670017])
@pytest.mark.parametrize("av,bv", [(9, 9), (9, 8)])
def test_field_boundary_worst_case(hip, m, av, bv):
    """Products run over F29 (p = 7 2^26 + 1) with coefficients as centered residues in [-8, 8]
    while 64 min(la, lb) <= (p - 1) / 2, i.e. min(la, lb) * 128 < p (min <= 3670016), and over
    BabyBear above (first at 3670017).  9 = -8 and 8 make every term +64 (9 x 9) or -64
    (9 x 8): the extreme sums c_i = +-64 min(i + 1, la, lb, la + lb - 1 - i) on both sides."""
    la, lb = m, m + 1000
    a = np.full(la, av, np.uint8)
    b = np.full(lb, bv, np.uint8)
    i = np.arange(la + lb - 1, dtype=np.int64)
    cnt = np.minimum(np.minimum(i + 1, la), np.minimum(lb, la + lb - 1 - i))
    want = ((av * bv) * cnt % 17).astype(np.uint8)
    nz = np.flatnonzero(want)
    want = want[:int(nz[-1]) + 1]
    assert hip.poly_mul(a, b) == want.tobytes()


# ---- batched products (plk_poly_mul_batch_dev: the prover's round-3 path) -------------------
def _trim(bts):
    bts = bts.rstrip(b"\x00")
    return bts if bts else b"\x00"


def _run_batch(hip, polys, spec):
    """spec: (ia, ib, acc) jobs over the operand pool; returns each job's untrimmed output"""
    import torch
    dev = torch.device("cuda:0")
    dp = [torch.from_numpy(p).to(dev) for p in polys]
    outs = [torch.full((len(polys[i]) + len(polys[j]) - 1,), 0xEE, dtype=torch.uint8, device=dev)
            for i, j, _ in spec]
    jobs = [(dp[i], len(polys[i]), dp[j], len(polys[j]), o, acc) for (i, j, acc), o in zip(spec, outs)]
    ws = hip.poly_mul_batch_workspace(jobs)
    work = torch.zeros(max(ws, 16), dtype=torch.uint8, device=dev)
    hip.poly_mul_batch_dev(jobs, work, ws, torch.cuda.current_stream())
    torch.cuda.synchronize()
    return [bytes(o.cpu().numpy()) for o in outs]


# lengths whose pairwise products all take 2^13-point transforms (plain and wrapped, e <= 16)
_POOL = [4097, 4100, 4096, 4000, 4099, 4090, 4097, 4100]


def test_batch_shared_operands(hip, oracle):
    """15 products of one size: two launch chunks (12 + 3), operands reused within and across
    the chunks, squarings, a repeated job (both operands shared: a fresh work array)."""
    polys = [np.frombuffer(gen.poly_inputs(40 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    spec = [(0, 1, 0), (0, 2, 0), (1, 2, 0), (0, 0, 0), (3, 4, 0), (4, 5, 0), (2, 5, 0), (1, 1, 0),
            (0, 3, 0), (2, 3, 0), (5, 5, 0), (1, 4, 0), (0, 1, 0), (3, 3, 0), (2, 4, 0)]
    outs = _run_batch(hip, polys, spec)
    for (i, j, _), out in zip(spec, outs):
        assert _trim(out) == oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), (i, j)


def test_batch_sum_group(hip, oracle):
    """a_0 a_1 + a_6 a_7 + a_0 a_7 (one shape, wrapped by 4) in one inverse transform"""
    polys = [np.frombuffer(gen.poly_inputs(60 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    spec = [(2, 3, 0), (0, 1, 0), (6, 7, 1), (0, 7, 1), (4, 5, 0)]
    outs = _run_batch(hip, polys, spec)
    full = len(polys[0]) + len(polys[1]) - 1

    def prod(i, j):
        p = np.frombuffer(oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), np.uint8).astype(np.int64)
        return np.pad(p, (0, full - len(p)))
    want = (prod(0, 1) + prod(6, 7) + prod(0, 7)) % 17
    assert outs[1] == want.astype(np.uint8).tobytes()
    assert outs[2] == b"\xEE" * full and outs[3] == b"\xEE" * full   # members' outputs untouched
    for k in (0, 4):
        i, j, _ = spec[k]
        assert _trim(outs[k]) == oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes())


def test_batch_group_across_launch_chunks(hip, oracle):
    """13 products with a sum group at positions 11-12: the batch is cut into launch chunks of at
    most 12 products at a group boundary (never inside a group)"""
    polys = [np.frombuffer(gen.poly_inputs(80 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    spec = [(k % 6, (k + 1) % 6, 0) for k in range(11)] + [(0, 1, 0), (6, 7, 1)]
    outs = _run_batch(hip, polys, spec)
    for k in range(11):
        i, j, _ = spec[k]
        assert _trim(outs[k]) == oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), k
    full = len(polys[0]) + len(polys[1]) - 1
    p1 = np.frombuffer(oracle.poly_mul(polys[0].tobytes(), polys[1].tobytes()), np.uint8).astype(np.int64)
    p2 = np.frombuffer(oracle.poly_mul(polys[6].tobytes(), polys[7].tobytes()), np.uint8).astype(np.int64)
    want = (np.pad(p1, (0, full - len(p1))) + np.pad(p2, (0, full - len(p2)))) % 17
    assert outs[11] == want.astype(np.uint8).tobytes()


def test_batch_small_workspace_and_bad_groups(hip, oracle):
    """a workspace of one product's size runs every product (and a 2-product group needs two);
    a member must follow a product of its transform size and at least its length"""
    import torch
    dev = torch.device("cuda:0")
    polys = [np.frombuffer(gen.poly_inputs(90 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    dp = [torch.from_numpy(p).to(dev) for p in polys]

    def run(spec, ws):
        outs = [torch.zeros(len(polys[i]) + len(polys[j]) - 1, dtype=torch.uint8, device=dev) for i, j, _ in spec]
        jobs = [(dp[i], len(polys[i]), dp[j], len(polys[j]), o, acc) for (i, j, acc), o in zip(spec, outs)]
        work = torch.zeros(ws, dtype=torch.uint8, device=dev)
        hip.poly_mul_batch_dev(jobs, work, ws, torch.cuda.current_stream())
        torch.cuda.synchronize()
        return [bytes(o.cpu().numpy()) for o in outs]

    one = hip.poly_mul_workspace(len(polys[0]), len(polys[1]))
    spec = [(0, 1, 0), (2, 3, 0), (4, 5, 0)]
    for (i, j, _), out in zip(spec, run(spec, one)):
        assert _trim(out) == oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes())
    with pytest.raises(Exception, match="sum group"):
        run([(0, 1, 0), (6, 7, 1)], one)                 # the group needs two products' workspace
    outs = run([(0, 1, 0), (6, 7, 1)], 2 * one)
    assert len(outs[0]) == len(polys[0]) + len(polys[1]) - 1
    with pytest.raises(Exception, match="does not follow"):
        run([(2, 3, 0), (0, 1, 1)], 2 * one)              # longer than the preceding job


# ---- blocked products: shapes beyond one transform's exact range --------------------------
# (min(la, lb) * 256 >= the BabyBear prime, or more than 2^27 output coefficients): the
# reference just runs its schoolbook loop; here they run as in-range piece products
# accumulated mod 17 (ntt.hip blocked_launch).
def _eval17(c):
    """c(x) mod 17 at x = 0..16 (x^i mod 17 has period 16 for x != 0)"""
    c = np.frombuffer(c, np.uint8) if isinstance(c, (bytes, bytearray)) else c
    c = c.astype(np.int64)
    s = np.concatenate([c, np.zeros((-len(c)) % 16, np.int64)]).reshape(-1, 16).sum(axis=0) % 17
    return [int(c[0] % 17)] + [int((s * np.array([pow(x, r, 17) for r in range(16)])).sum() % 17)
                               for x in range(1, 17)]


@pytest.mark.parametrize("la,lb", [(20000, 15000), (12345, 999), (50000, 50001), (3001, 7000)])
def test_blocked_forced_vs_oracle(hip, oracle, la, lb):
    """The blocked path with small pieces (PLK_OPT_POLY_BLOCK_L/_S) against the oracle's NTT."""
    a, b = gen.poly_inputs(77 + la, la, lb)
    with hip.options(POLY_BLOCK_L=3001, POLY_BLOCK_S=1000):
        got = hip.poly_mul(a, b)
    assert got == oracle.poly_mul_ntt(a, b)


def test_blocked_forced_device_api(hip, oracle):
    import torch
    la, lb = 30000, 2100
    a, b = gen.poly_inputs(5, la, lb)
    dev = torch.device("cuda:0")
    da, db = torch.from_numpy(np.frombuffer(a, np.uint8).copy()).to(dev), torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to(dev)
    out = torch.full((la + lb - 1,), 0xEE, dtype=torch.uint8, device=dev)
    nz = torch.zeros(4, dtype=torch.int32, device=dev)
    with hip.options(POLY_BLOCK_L=4096, POLY_BLOCK_S=513):
        work = torch.zeros(max(16, hip.poly_mul_workspace(la, lb)), dtype=torch.uint8, device=dev)
        hip.poly_mul_dev(da, la, db, lb, out, nz, work, torch.cuda.current_stream())
        torch.cuda.synchronize()
    n = int(nz[0].item()) or 1
    assert bytes(out[:n].cpu().numpy()) == oracle.poly_mul_ntt(a, b)


def test_blocked_beyond_babybear_range(hip, oracle):
    """8,000,000 x 8,000,000 (min * 256 >= 15 2^27 + 1: no single transform is exact): every
    byte equals the oracle's product -- an independent blocked decomposition (both operands in
    pieces, NTTs over 998244353, orc_poly_mul_ntt_blocked, itself checked against the schoolbook
    restatement in tests/test_oracle_cpu.py; ~8 s of host time) -- and, as size-independent
    properties, the product at all 17 points of GF(17) equals a(x) b(x) and the lowest / highest
    3000 coefficients equal the products of the operands' first / last 3000 coefficients.  The
    reference itself cannot be run at this size (its schoolbook loop would take days)."""
    la = lb = 8_000_000
    a, b = gen.poly_inputs(8008, la, lb)
    got = hip.poly_mul(a, b)
    rl = la + lb - 1
    full = np.zeros(rl, np.uint8)
    full[:len(got)] = np.frombuffer(got, np.uint8)
    ea, eb, ec = _eval17(a), _eval17(b), _eval17(full)
    assert ec == [(x * y) % 17 for x, y in zip(ea, eb)]
    t = 3000
    lo = np.frombuffer(oracle.poly_mul_ntt(a[:t], b[:t]), np.uint8)
    assert np.array_equal(full[:t], np.pad(lo, (0, max(0, t - len(lo))))[:t])
    hi = np.frombuffer(oracle.poly_mul_ntt(a[-t:], b[-t:]), np.uint8)
    hi = np.pad(hi, (0, 2 * t - 1 - len(hi)))
    assert np.array_equal(full[rl - t:], hi[t - 1:])
    assert got == oracle.poly_mul_ntt(a, b)


@pytest.mark.parametrize("mode", [0, 2])
def test_batch_shared_operands_fix_modes(hip, oracle, mode):
    """The batch of test_batch_shared_operands with the shared operands' separate lo = 0 pass off
    (PLK_OPT_NTT_SHARED_FIX = 0: every center item transforms its operands) and forced (2)."""
    polys = [np.frombuffer(gen.poly_inputs(40 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    spec = [(0, 1, 0), (0, 2, 0), (1, 2, 0), (0, 0, 0), (3, 4, 0), (4, 5, 0), (2, 5, 0), (0, 1, 0),
            (6, 7, 1), (0, 7, 1), (5, 5, 0), (1, 4, 0), (1, 1, 0), (3, 3, 0), (2, 4, 0)]
    with hip.options(NTT_SHARED_FIX=mode):
        got = [_trim(out).hex() for out in _run_batch(hip, polys, spec)]
    full = len(polys[6]) + len(polys[7]) - 1

    def prod(i, j):
        p = np.frombuffer(oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), np.uint8).astype(np.int64)
        return np.pad(p, (0, full - len(p)))
    for k, (i, j, acc) in enumerate(spec):
        if k == 7:   # sum group leader: a_0 a_1 + a_6 a_7 + a_0 a_7
            want = _trim(((prod(0, 1) + prod(6, 7) + prod(0, 7)) % 17).astype(np.uint8).tobytes())
        elif acc:
            continue
        else:
            want = oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes())
        assert bytes.fromhex(got[k]) == want, (mode, k)


@pytest.mark.parametrize("csum", [0, 1])
def test_batch_center_sum_member_pair_first(hip, oracle, csum):
    """A sum group whose only pair with both operands still to transform is a member's (a_6 a_7;
    a_0 is shared with a later job, so its lo = 0 pass runs once beforehand): merged into the
    leader's center item (PLK_OPT_NTT_CENTER_SUM = 1, the member's pair taking the leader's
    place) or added in the inverse pass (0).  Same bytes either way."""
    polys = [np.frombuffer(gen.poly_inputs(120 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    spec = [(0, 1, 0), (6, 7, 1), (0, 4, 0), (2, 3, 0)]
    with hip.options(NTT_CENTER_SUM=csum):
        outs = _run_batch(hip, polys, spec)
    full = len(polys[0]) + len(polys[1]) - 1

    def prod(i, j):
        p = np.frombuffer(oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), np.uint8).astype(np.int64)
        return np.pad(p, (0, full - len(p)))
    assert outs[0] == ((prod(0, 1) + prod(6, 7)) % 17).astype(np.uint8).tobytes()
    assert outs[1] == b"\xEE" * full
    for k in (2, 3):
        i, j, _ = spec[k]
        assert _trim(outs[k]) == oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), k


def test_batch_center_schedule_2_19(hip, oracle):
    """Ten 2^18 x 2^18 products (2^19-point transforms: 128 tiles per product, 10 x 128 center
    items on 512 resident blocks) with shared operands and a merged 3-product sum group, so the
    items carry 1..5 lo = 0 passes and the center's slot order balances them over the blocks'
    four item sets (center_schedule).  Every product against the oracle's NTT product."""
    n = 1 << 18
    polys = [np.frombuffer(gen.poly_inputs(140 + i, n, 1)[0], np.uint8) for i in range(9)]
    spec = [(0, 1, 0), (2, 3, 1), (4, 5, 1), (0, 2, 0), (0, 0, 0), (1, 4, 0), (6, 7, 0), (7, 8, 0), (3, 6, 0),
            (5, 8, 0)]
    outs = _run_batch(hip, polys, spec)
    full = 2 * n - 1

    def prod(i, j):
        p = np.frombuffer(oracle.poly_mul_ntt(polys[i].tobytes(), polys[j].tobytes()), np.uint8).astype(np.int64)
        return np.pad(p, (0, full - len(p)))
    want0 = (prod(0, 1) + prod(2, 3) + prod(4, 5)) % 17
    assert outs[0] == want0.astype(np.uint8).tobytes()
    for k in range(3, len(spec)):
        i, j, _ = spec[k]
        assert _trim(outs[k]) == oracle.poly_mul_ntt(polys[i].tobytes(), polys[j].tobytes()), k


@pytest.mark.parametrize("csum", [0, 1])
def test_batch_sum_group_mixed_shapes(hip, oracle, csum):
    """A sum group of one transform size (2^13) with shorter members: a_0 a_1 (8196 coefficients,
    wrapped by 4) + a_2 a_3 (8095, not wrapped) + a_6 a_4 (8195, wrapped by 3) -- the wrapped top
    coefficients come from each product's own operand lengths.  A member longer than its leader
    is refused."""
    polys = [np.frombuffer(gen.poly_inputs(160 + i, n, 1)[0], np.uint8) for i, n in enumerate(_POOL)]
    spec = [(5, 5, 0), (0, 1, 0), (2, 3, 1), (6, 4, 1)]
    with hip.options(NTT_CENTER_SUM=csum):
        outs = _run_batch(hip, polys, spec)
    full = len(polys[0]) + len(polys[1]) - 1

    def prod(i, j):
        p = np.frombuffer(oracle.poly_mul(polys[i].tobytes(), polys[j].tobytes()), np.uint8).astype(np.int64)
        return np.pad(p, (0, full - len(p)))
    assert outs[1] == ((prod(0, 1) + prod(2, 3) + prod(6, 4)) % 17).astype(np.uint8).tobytes()
    assert _trim(outs[0]) == oracle.poly_mul(polys[5].tobytes(), polys[5].tobytes())
    with pytest.raises(Exception, match="does not follow"):
        _run_batch(hip, polys, [(2, 3, 0), (0, 1, 1)])


@pytest.mark.parametrize("opts", [{"NTT_F29": 0}, {"NTT_SHARE": 0}, {"NTT_SHARED_FIX": 0}, {"NTT_SHARED_FIX": 2},
                                  {"NTT_CENTER_BLOCKS": 300}, {"NTT_CENTER_SUM": 0}, {"NTT_TABLE_SHARE": 0},
                                  {"POLY_BLOCK_L": 1 << 18, "POLY_BLOCK_S": 1 << 16}])
def test_option_sweep(hip, oracle, opts):
    """Each poly_mul switch (PLK_OPT_*) off its default: BabyBear for every product, no shared
    operands, the shared-operand pass off / forced, a centre grid that does not divide the items,
    no centre sum groups, per-array column reads, forced blocked pieces -- the C3-size reference
    digests and the batch cases (shared operands across launch chunks, sum groups) unchanged."""
    with hip.options(**opts):
        for idx in range(3):
            test_golden_c3_size_digests(hip, idx)
        test_batch_shared_operands(hip, oracle)
        test_batch_sum_group(hip, oracle)
        test_batch_group_across_launch_chunks(hip, oracle)
