"""GPU parity for the ops around the hot path through the C ABI, against
outputs recorded from the compiled reference (tests/golden/polyops.json, poly_next.json):
poly_divide (src/poly.h:124-177), poly_eval (src/poly.h:265-272), matrix_mul / matrix_inv
(src/matrix.h:79-176, plonk_new's Vandermonde inverse src/plonk.h:105-113) and
interpolate_at_h (src/plonk.h:162-195).  Bytes must be identical, raw HF bytes included."""
import numpy as np
import pytest

import gen
from conftest import load_golden
from make_golden import big_division_inputs

pytestmark = pytest.mark.gpu


def test_divide_goldens(hip):
    for c in load_golden("polyops.json")["divide"] + load_golden("poly_next.json")["divide"]:
        q, r = hip.poly_divide(bytes.fromhex(c["num"]), bytes.fromhex(c["den"]))
        assert (q.hex(), r.hex()) == (c["q"], c["r"]), c.get("note", c["den"])


@pytest.mark.parametrize("idx", range(7))
def test_divide_big_goldens(hip, idx):
    c = load_golden("polyops.json")["divide_big"][idx]
    a, b = big_division_inputs(c["seed"], c["nl"], c["kind"], c["param"])
    q, r = hip.poly_divide(a, b)
    assert (len(q), len(r)) == (c["ql"], c["rl"])
    assert gen.digest(np.frombuffer(q, np.uint8)) == c["q_sha256"]
    assert gen.digest(np.frombuffer(r, np.uint8)) == c["r_sha256"]


def test_divide_vs_oracle_random(hip, oracle):
    """random shapes over every path (constant, linear, binomial short / long chains, general,
    raw numerator bytes) against the oracle restatement (itself pinned to the reference)"""
    rng = np.random.default_rng(11)
    for t in range(150):
        kind = t % 5
        nl = int(rng.integers(1, 9000 if kind != 3 else 300))
        num = rng.integers(0, 17, nl).astype(np.uint8)
        if kind == 0:
            den = np.array([int(rng.integers(1, 17))], np.uint8)
        elif kind == 1:
            den = np.array([int(rng.integers(0, 17)), int(rng.integers(1, 17))], np.uint8)
        elif kind == 2:
            m = int(rng.integers(2, 40))
            den = np.zeros(m + 1, np.uint8)
            den[0], den[m] = int(rng.integers(0, 17)), int(rng.integers(1, 17))
        elif kind == 3:
            den = rng.integers(0, 17, int(rng.integers(2, 12))).astype(np.uint8)
            den[-1] = max(int(den[-1]), 1)
        else:
            den = np.array([int(rng.integers(0, 17)), 1], np.uint8)
            num[rng.integers(0, nl, 3)] = rng.integers(17, 256, 3)
        q, r = hip.poly_divide(num, den)
        assert (q, r) == oracle.poly_divide(num, den), (kind, nl, den.tolist())


def test_divide_errors(hip):
    with pytest.raises(hip.PlonkHipError, match="Division by zero polynomial"):
        hip.poly_divide([1, 2, 3], [0, 0])
    with pytest.raises(hip.PlonkHipError) as e:
        hip.poly_divide([1, 2, 3], [1, 20])
    assert e.value.code == hip.PLK_ERR_RANGE


def test_divide_device_api(hip):
    import torch
    a, _ = gen.poly_inputs(0x515, 1 << 16, 1)
    den = np.array([12, 1], np.uint8)
    d_num = torch.from_numpy(a.copy()).cuda()
    q = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    r = torch.zeros(16, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(2, dtype=torch.int32, device="cuda")
    work = torch.zeros(hip.poly_divide_workspace(a.size, 2), dtype=torch.uint8, device="cuda")
    hip.poly_divide_dev(d_num, a.size, den, q, r, lens, work)
    torch.cuda.synchronize()
    wq, wr = hip.poly_divide(a, den)
    ql, rl = lens.cpu().tolist()
    assert bytes(q.cpu().numpy()[:max(ql, 1)]) == wq and bytes(r.cpu().numpy()[:max(rl, 1)]) == wr


def test_eval_goldens(hip):
    cases = load_golden("polyops.json")["eval"] + load_golden("poly_next.json")["eval"]
    for c in cases:
        assert hip.poly_eval(bytes.fromhex(c["p"]), c["x"]) == c["y"], c.get("note")
    ys = hip.poly_eval_batch([bytes.fromhex(c["p"]) for c in cases[:70]], [c["x"] for c in cases[:70]])
    assert ys == [c["y"] for c in cases[:70]]


def test_eval_vs_oracle_large_and_raw(hip, oracle):
    rng = np.random.default_rng(5)
    polys, xs = [], []
    for L in (1 << 20, (1 << 20) + 7, 65536, 3):
        for raw in (False, True):
            p = rng.integers(0, 17, L).astype(np.uint8)
            if raw:
                p[int(rng.integers(0, L))] = 248
            polys.append(p)
            xs.append(int(rng.integers(0, 256)))
    ys = hip.poly_eval_batch(polys, xs)
    assert ys == [oracle.poly_eval(p, x) for p, x in zip(polys, xs)]


def test_eval_device_api(hip, oracle):
    import torch
    rng = np.random.default_rng(9)
    hs = [rng.integers(0, 17, L).astype(np.uint8) for L in (5, 100000, 1 << 18)]
    ds = [torch.from_numpy(h).cuda() for h in hs]
    ys = torch.zeros(3, dtype=torch.uint8, device="cuda")
    tick = torch.zeros(hip.poly_eval_workspace(3), dtype=torch.uint8, device="cuda")
    for rep in range(2):   # the workspace is re-armed by the launch
        hip.poly_eval_batch_dev(ds, [h.size for h in hs], [4, 13, 16], ys, tick)
        torch.cuda.synchronize()
        assert ys.cpu().tolist() == [oracle.poly_eval(h, x) for h, x in zip(hs, (4, 13, 16))]


def test_matrix_goldens(hip):
    g = load_golden("polyops.json")
    for c in g["matrix_inv"]:
        assert hip.matrix_inv(bytes.fromhex(c["m"]), c["n"]).hex() == c["inv"], c["note"]
    for c in g["matrix_mul"]:
        assert hip.matrix_mul(bytes.fromhex(c["a"]), c["m"], c["k"], bytes.fromhex(c["b"]), c["n"]).hex() == c["out"]


def test_plonk_new_vandermonde_and_interpolate(hip):
    """plonk_new's h_pows_inv (src/plonk.h:105-113) rebuilt on the GPU from H equals the
    reference's; interpolate_at_h through it equals the reference's (ref_interpolate4)"""
    g = load_golden("prove.json")
    setup = g["setups"]["0"]
    h = bytes.fromhex(setup["h"])
    n = len(h)
    vander = bytes(pow(h[r], c, 17) for r in range(n) for c in range(n))
    h_inv = hip.matrix_inv(vander, n)
    assert h_inv.hex() == setup["h_pows_inv"]
    for c in g["interpolate_at_h"]:
        assert hip.interpolate(h_inv, c["values"]).hex() == c["out"]


@pytest.mark.parametrize("kind", ["raw_binomial", "general"])
def test_divide_device_api_exact_buffers(hip, oracle, kind):
    """The reference's loop on the device (non-canonical numerator bytes behind the binomial
    chain scans, or a divisor with middle terms) writes ONLY the documented sizes: quot
    nl - dl + 1 bytes, rem min(dl - 1, nl) bytes (the running remainder lives in the workspace);
    guard bytes after both buffers stay intact."""
    import torch
    nl = 3000
    num, _ = gen.poly_inputs(0x77 + len(kind), nl, 1)
    num = num.copy()
    if kind == "raw_binomial":
        num[nl // 2] = 200                                # not a GF(17) value: the gated loop runs
        den = np.zeros(65, np.uint8)
        den[0], den[64] = 16, 1                           # x^64 - 1
    else:
        den = np.array([3, 0, 5, 0, 0, 1], np.uint8)      # middle terms: the loop always runs
    dl = den.size
    ql, rl = nl - dl + 1, min(dl - 1, nl)
    G = 64
    q = torch.full((ql + G,), 0xEE, dtype=torch.uint8, device="cuda")
    r = torch.full((rl + G,), 0xEE, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(2, dtype=torch.int32, device="cuda")
    work = torch.zeros(hip.poly_divide_workspace(nl, dl), dtype=torch.uint8, device="cuda")
    hip.poly_divide_dev(torch.from_numpy(num).cuda(), nl, den, q, r, lens, work)
    torch.cuda.synchronize()
    qh, rh = q.cpu().numpy(), r.cpu().numpy()
    assert (qh[ql:] == 0xEE).all() and (rh[rl:] == 0xEE).all()
    wq, wr = hip.poly_divide(num, den)                    # host form (pinned to goldens above)
    oq, orr = oracle.poly_divide(num, den)
    assert wq == oq and wr.rstrip(b"\x00") == orr.rstrip(b"\x00")
    lq, lr = lens.cpu().tolist()
    assert bytes(qh[:max(lq, 1)]) == wq and bytes(rh[:max(lr, 1)]) == wr


def _tiny_cases(seed):
    """host-call shapes on both sides of the 16 KiB toy-size path (capi.hip tiny_ok): evaluations
    in batches over 12 (several launches), empty and raw-byte (>= 240: the reference-loop re-run)
    polynomials, short-operand products with raw bytes and trailing cancellation"""
    rng = np.random.default_rng(seed)
    evals = []
    for t in range(6):
        n = int(rng.integers(1, 30))
        polys = []
        for _ in range(n):
            ln = int(rng.integers(0, 3000 if t < 4 else 9000))
            p = rng.integers(0, 17 if t % 2 else 256, ln).astype(np.uint8)
            polys.append(p)
        evals.append((polys, rng.integers(0, 256, n).astype(np.uint8)))
    muls = []
    for t in range(40):
        la = int(rng.integers(1, 33))
        lb = int(rng.integers(1, 20000 if t % 3 == 0 else 3000))
        a = rng.integers(0, 17 if t % 2 else 256, la).astype(np.uint8)
        b = rng.integers(0, 17, lb).astype(np.uint8)
        if t % 5 == 0:
            b[-1] = 0   # trailing zero: the trimmed length comes from the trim pass
        muls.append((a, b) if t % 4 else (b, a))
    return evals, muls


def test_toy_size_calls_vs_oracle(hip, oracle):
    evals, muls = _tiny_cases(5)
    for polys, xs in evals:
        got = hip.poly_eval_batch(polys, xs)
        assert list(got) == [oracle.poly_eval(p, x) for p, x in zip(polys, xs)]
    for a, b in muls:
        assert hip.poly_mul(a, b) == oracle.poly_mul(a, b), (len(a), len(b))


def test_toy_size_path_matches_staged_path(hip):
    """PLK_OPT_TINY_CALLS = 0 (every host call staged through device copies) gives the same
    bytes as the mapped-memory path"""
    want = _child_digest(hip)
    with hip.options(TINY_CALLS=0):
        got = _child_digest(hip)
    assert got == want


def _child_digest(h):
    import hashlib
    evals, muls = _tiny_cases(9)
    m = hashlib.sha256()
    for polys, xs in evals:
        m.update(bytes(h.poly_eval_batch(polys, xs)))
    for a, b in muls:
        m.update(h.poly_mul(a, b))
    return m.hexdigest()
