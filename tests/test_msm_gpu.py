"""GPU parity for the MSM (srs_eval_at_s, reference src/srs.h:53-68) through the C ABI.

Bit-exact on the 3-byte G1 {x, y, infinite} against (a) golden vectors recorded from the
compiled reference and (b) the oracle's serial fold / discrete-log checker on seeded inputs.
"""
import numpy as np
import pytest

import gen
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _bytes(h):
    return np.frombuffer(bytes.fromhex(h), np.uint8)


def test_golden_small_cases(hip):
    g = load_golden("msm.json")
    for c in g["cases"]:
        pts, sc = _bytes(c["points"]), _bytes(c["scalars"])
        assert hip.msm_g1(pts, sc).hex() == c["out"], (c["kind"], c["n"])


def test_golden_irregular_encodings(hip):
    """off-curve points, coordinates >= 101, flagged identities with coordinates: the
    reference folds them with raw formulas; the GPU must reproduce it byte for byte."""
    g = load_golden("msm.json")
    for c in g["irregular"]:
        pts, sc = _bytes(c["points"]), _bytes(c["scalars"])
        assert hip.msm_g1(pts, sc).hex() == c["out"], (c["n"], c["bad"])


@pytest.mark.parametrize("idx", range(8))
def test_golden_large_seeded(hip, idx):
    g = load_golden("msm.json")
    c = g["large"][idx]
    pts, sc = gen.msm_inputs(c["seed"], c["n"], c["kind"])
    assert hip.msm_g1(pts, sc).hex() == c["out"], (c["kind"], c["n"])


def test_survey_known_answers(hip, oracle):
    g = load_golden("msm.json")
    for c in g["survey_xorshift"]:
        pts, sc = oracle.gen_survey_msm(c["n"])
        assert hip.msm_g1(pts, sc).hex() == c["out"]


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 255, 256, 4095, 4096, 4097, 65535,
                               (1 << 16) + 13, 1 << 18])
@pytest.mark.parametrize("kind", ["subgroup", "full", "bytes"])
def test_sizes_vs_oracle_fold(hip, oracle, n, kind):
    pts, sc = gen.msm_inputs(0x5EED + n, n, kind)
    assert hip.msm_g1(pts, sc) == oracle.msm(pts, sc)


def test_all_zero_scalars_and_all_identity(hip):
    pts, _ = gen.msm_inputs(3, 5000, "full")
    assert hip.msm_g1(pts, np.zeros(5000, np.uint8)) == bytes([0, 0, 1])
    ident = np.tile(np.array([0, 0, 1], np.uint8), 5000)
    assert hip.msm_g1(ident, np.full(5000, 7, np.uint8)) == bytes([0, 0, 1])


def test_two_torsion_point(hip, oracle):
    # (48, 0) has order 2: odd scalar sums give (48, 0), even give the identity
    pts = np.tile(np.array([48, 0, 0], np.uint8), 101)
    for k in (1, 2, 3, 16):
        sc = np.full(101, k, np.uint8)
        assert hip.msm_g1(pts, sc) == oracle.msm(pts, sc)


def test_irregular_late_in_large_input(hip, oracle):
    n = 20000
    pts, sc = gen.msm_inputs(0xBAD, n, "full")
    pts = pts.copy()
    pts[n - 7] = (3, 3, 0)          # off-curve near the end
    sc[n - 7] = 5
    assert hip.msm_g1(pts, sc) == oracle.msm(pts, sc)
    pts[123] = (0, 0, 2)            # non-boolean flag byte
    assert hip.msm_g1(pts, sc) == oracle.msm(pts, sc)


@pytest.mark.parametrize("where", ["first", "chunk_edge", "last"])
def test_irregular_in_2_22_points(hip, oracle, where):
    """one irregular point in a 2^22-point input: the prefix before it is summed in parallel,
    the raw fold runs from it (reference fold, src/srs.h:59-66); before, every point of the
    input went through one GPU lane"""
    c = load_golden("msm.json")["large"][7]
    pts, sc = gen.msm_inputs(c["seed"], c["n"], c["kind"])
    pts = pts.copy()
    idx = {"first": 0, "chunk_edge": 16384 * 3 - 1, "last": c["n"] - 1}[where]
    pts[idx] = (5, 5, 0)
    sc = sc.copy()
    sc[idx] = 3
    assert hip.msm_g1(pts, sc) == oracle.msm(pts, sc)


def _serial_dev(hip, pts, sc):
    """plk_msm_g1_serial_dev (the exact raw fold) on device copies; returns (bytes, seconds)"""
    import time
    import torch
    dev = torch.device("cuda:0")
    dp = torch.from_numpy(np.ascontiguousarray(pts).reshape(-1).copy()).to(dev)
    ds = torch.from_numpy(np.ascontiguousarray(sc).copy()).to(dev)
    res = torch.zeros(hip.MSM_RESULT_BYTES, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hip.msm_g1_serial_dev(dp, ds, sc.size, res, st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g = hip.MSM_G1_OFFSET
    return bytes(res[g:g + 3].cpu().numpy()), dt


def _raw_points(seed, n, frac_bad):
    """subgroup points with a fraction replaced by raw byte triples of every irregular shape:
    off-curve canonical coordinates, coordinates >= 101, flag bytes 1 / 2 / 255 with coordinates"""
    pts, sc = gen.msm_inputs(seed, n, "bytes")
    pts = pts.copy()
    rng = np.random.default_rng(seed)
    bad = rng.random(n) < frac_bad
    m = int(bad.sum())
    raw = rng.integers(0, 256, (m, 3)).astype(np.uint8)
    shape = rng.integers(0, 4, m)
    raw[shape == 0] %= 101
    raw[shape == 0, 2] = 0
    raw[shape == 1, 2] = 0
    raw[shape == 2, 2] = rng.choice([1, 2, 255], int((shape == 2).sum()))
    raw[shape == 3, 2] = 1
    pts[bad] = raw
    return pts, sc


@pytest.mark.parametrize("n,frac", [(8192, 1.0), (9001, 0.01), (20000, 0.3), (65536, 0.001), (100003, 1.0),
                                    (300000, 0.05)])
def test_chunked_fold_vs_oracle(hip, oracle, n, frac):
    """The chunked raw fold (msm_fold_*_kernel: every chunk a map over the 10,202 canonical
    accumulator states, resolved in order) against the oracle's serial fold, from inputs that are
    raw everywhere to a few irregular points; sizes on and off the chunk grid."""
    pts, sc = _raw_points(n + int(frac * 1000), n, frac)
    got, _ = _serial_dev(hip, pts, sc)
    assert got == oracle.msm(pts, sc)
    assert hip.msm_g1(pts, sc) == got


@pytest.mark.parametrize("case", ["identity_runs", "raw_inf_runs", "zero_scalars", "offcurve_after_prefix"])
def test_chunked_fold_state_edges(hip, oracle, case):
    """Inputs that keep raw accumulator states alive across chunk boundaries (infinite terms
    pass the accumulator through unchanged; a raw term on an infinite accumulator becomes it)
    and a long canonical prefix before the first irregular point."""
    n = 70000
    pts, sc = gen.msm_inputs(77, n, "full")
    pts, sc = pts.copy(), sc.copy()
    if case == "identity_runs":       # raw (coordinates >= 101) term, then long runs of identities
        pts[::5000] = (200, 150, 0)
        sc[::5000] = 1
        for s0 in range(1, n, 5000):
            pts[s0:s0 + 3000] = (0, 0, 1)
    elif case == "raw_inf_runs":      # flagged points with coordinates, scalar 1: terms are the raw bytes
        pts[1::3] = (9, 250, 1)
        sc[1::3] = 1
        pts[2::7] = (0, 0, 1)
    elif case == "zero_scalars":      # irregular points whose terms are the identity (scalar 0)
        pts[::2] = (7, 7, 0)
        sc[::2] = 0
    else:
        pts[n - 20000] = (3, 3, 0)
        sc[n - 20000] = 2
    got, _ = _serial_dev(hip, pts, sc)
    assert got == oracle.msm(pts, sc), case


@pytest.mark.parametrize("kind", ["first_flagged", "all_raw"])
def test_irregular_2_22_beats_reference_cpu(hip, oracle, kind):
    """The worst cases of the raw fold at 2^22 points -- the first point irregular, so every
    addition is order-dependent, and every point a raw byte triple -- must finish faster than
    the reference's own srs_eval_at_s (oracle/_ref: the unmodified reference, gcc -O2) on this
    host for the same input, and give its bytes."""
    from pyoracle import Reference
    c = load_golden("msm.json")["large"][7]
    if kind == "first_flagged":
        pts, sc = gen.msm_inputs(c["seed"], c["n"], c["kind"])
        pts = pts.copy()
        pts[0] = (7, 7, 1)                              # identity flag with coordinates
    else:
        pts, sc = _raw_points(99, c["n"], 1.0)
    _serial_dev(hip, pts[:20000], sc[:20000])           # warm
    got, dt = _serial_dev(hip, pts, sc)
    assert Reference.available(), "oracle/_ref/libplonkref.so missing (built where /root/reference exists)"
    import time
    R = Reference()
    t0 = time.perf_counter()
    want = R.msm(pts, sc)
    ref_s = time.perf_counter() - t0
    print("raw fold 2^22 (%s): device %.4f s, reference CPU %.3f s" % (kind, dt, ref_s))
    assert got == want
    assert dt < ref_s, (dt, ref_s)


def test_srs_eval_degree_check(hip):
    pts = np.tile(np.array([1, 2, 0], np.uint8), 4)
    with pytest.raises(ValueError):
        hip.srs_eval_at_s(pts, np.ones(5, np.uint8))
    assert hip.srs_eval_at_s(pts, np.array([1, 1, 0], np.uint8)) == bytes([68, 74, 0])


def test_device_api_relaunch_and_unaligned(hip, oracle):
    """plk_msm_g1_dev: the result record re-arms itself between launches; misaligned
    device pointers take the byte path."""
    import torch
    dev = torch.device("cuda:0")
    n = 100003
    pts, sc = gen.msm_inputs(77, n, "full")
    want = oracle.msm(pts, sc)
    dp = torch.zeros(3 * n + 64, dtype=torch.uint8, device=dev)
    ds = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    res = torch.zeros(hip.MSM_RESULT_BYTES, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    hip.msm_result_init(res, st)
    for off in (0, 0, 1, 5):
        dp[off * 3:off * 3 + 3 * n] = torch.from_numpy(pts.reshape(-1)).to(dev)
        ds[off:off + n] = torch.from_numpy(sc).to(dev)
        hip.msm_g1_dev(dp.data_ptr() + 3 * off, ds.data_ptr() + off, n, res, st)
        torch.cuda.synchronize()
        r = hip.parse_result(res.cpu().numpy())
        assert r["irregular"] == 0
        assert r["g1"] == want, off
        _, lg = None, oracle.msm_dlog(pts, sc)[0]
        assert r["log"] == lg


def test_combine_partials(hip, oracle):
    """point-range shards -> partial logs -> sum -> EXP: the multi-GPU reduction path."""
    import torch
    dev = torch.device("cuda:0")
    n = 1 << 16
    pts, sc = gen.msm_inputs(91, n, "full")
    shards = 4
    logs = []
    for s in range(shards):
        a, b = s * n // shards, (s + 1) * n // shards
        lg, _ = oracle.msm_dlog(pts[a:b], sc[a:b])
        logs.append(lg)
    dl = torch.tensor(logs, dtype=torch.int32, device=dev)
    out = torch.zeros(4, dtype=torch.uint8, device=dev)
    hip.msm_combine_dev(dl, shards, out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()[:3]) == oracle.msm(pts, sc)


# launch-geometry switches (PLK_OPT_MSM_*), alone and combined; {} = the built-in choice
_GEOM = [{}, {"MSM_THREADS": 256}, {"MSM_THREADS": 1024}, {"MSM_MAX_BLOCKS": 64}, {"MSM_MAX_BLOCKS": 1000},
         {"MSM_GROUPS": 1}, {"MSM_GROUPS": 4}, {"MSM_COPIES": 1}, {"MSM_HALF": 0},
         {"MSM_HALF": 0, "MSM_THREADS": 1024, "MSM_GROUPS": 4, "MSM_COPIES": 1}]


def test_geometry_options_vs_golden(hip, oracle):
    """Every MSM launch-geometry switch (threads per block, resident blocks, groups in flight, table
    copies, half groups) gives the recorded reference results: single device launches on the
    golden seeded inputs (up to 2^22 points) and a ragged length against the oracle, and the batched
    launch (the headline kernel) on 5 inputs of 2^20 + 16 points (aligned rows) and of 2^20 + 7
    (byte-wise rows) against the oracle."""
    import torch
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    g = load_golden("msm.json")
    cases = [(c["out"], gen.msm_inputs(c["seed"], c["n"], c["kind"])) for c in g["large"]]
    pts, sc = gen.msm_inputs(79, 1000003, "full")
    cases.append((oracle.msm(pts, sc).hex(), (pts, sc)))
    dcases = [(w, torch.from_numpy(p.reshape(-1)).to(dev), torch.from_numpy(s).to(dev), len(s)) for w, (p, s) in cases]
    res = torch.zeros(hip.MSM_RESULT_BYTES, dtype=torch.uint8, device=dev)
    hip.msm_result_init(res, st)
    batch, R = 5, hip.MSM_RESULT_BYTES
    bres = torch.zeros(batch * R, dtype=torch.uint8, device=dev)
    for i in range(batch):
        hip.msm_result_init(bres[i * R:(i + 1) * R], st)
    batches = []
    for nb in ((1 << 20) + 16, (1 << 20) + 7):
        bp, bs = gen.msm_inputs(nb % 97, nb * batch, "full")
        want_b = [oracle.msm(bp[i * nb:(i + 1) * nb], bs[i * nb:(i + 1) * nb]) for i in range(batch)]
        batches.append((nb, torch.from_numpy(bp.reshape(-1)).to(dev), torch.from_numpy(bs).to(dev), want_b))
    for opts in _GEOM:
        with hip.options(**opts):
            for want, dp, ds, n in dcases:
                hip.msm_g1_dev(dp, ds, n, res, st)
                torch.cuda.synchronize()
                assert hip.parse_result(res.cpu().numpy())["g1"].hex() == want, (opts, n)
            for nb, bpd, bsd, want_b in batches:
                hip.msm_g1_batch_dev(bpd, 3 * nb, bsd, nb, nb, batch, bres, st)
                torch.cuda.synchronize()
                got = bres.cpu().numpy()
                for i in range(batch):
                    assert hip.parse_result(got[i * R:(i + 1) * R])["g1"] == want_b[i], (opts, nb, i)
