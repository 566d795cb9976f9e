"""Device prover (plk_prover_*, plonk.c_amd/csrc/prove.hip) against the reference prover.

* n = 4: every proof the compiled reference produced (tests/golden/prove.json, 26 instances,
  two SRS kinds) is reproduced byte for byte by plk_prover_prove, and every instance the
  reference rejects (failed assert, exit) is rejected.
* larger n: rounds 1-5 from synthetic interpolated polynomials (prove-shaped, non-strict:
  GF(17) has no subgroup of that order, so no satisfiable circuit exists) against the CPU
  restatement oracle/prove_ref.py, which is itself pinned to the same fixtures
  (tests/test_prove_cpu.py).
"""
import numpy as np
import pytest
import torch

import gen
from conftest import load_golden
from prove_ref import Prover as RefProver, ProveError

pytestmark = pytest.mark.gpu


def _setup(g, case):
    key = "short" if case["srs_n"] == 4 else str(case["srs_mode"])
    return {k: bytes.fromhex(v) for k, v in g["setups"][key].items()}


def _circuit(case):
    gt, cp, w = case["gates"], case["copies"], case["wires"]
    return dict(q_m=gt[0:4], q_l=gt[4:8], q_r=gt[8:12], q_o=gt[12:16], q_c=gt[16:20],
                copy_a=cp[0:8], copy_b=cp[8:16], copy_c=cp[16:24], a=w[0:4], b=w[4:8], c=w[8:12])


def test_prove_fixture_proofs(hip):
    g = load_golden("prove.json")
    provers = {}
    for case in g["proofs"]:
        key = (case["srs_n"], case["srs_mode"])
        if key not in provers:
            s = _setup(g, case)
            provers[key] = hip.Prover(4, s["z_h"], s["g1s"], s["h"], s["k1_h"], s["k2_h"], s["h_pows_inv"])
        got = provers[key].prove(**_circuit(case), chal=case["chal"], rand=case["rand"])
        assert got.hex() == case["proof"], (case["chal"], case["rand"], case["srs_mode"])


def test_prove_rejects_what_the_reference_rejects(hip):
    g = load_golden("prove.json")
    for case in g["failures"]:
        s = _setup(g, case)
        pr = hip.Prover(4, s["z_h"], s["g1s"], s["h"], s["k1_h"], s["k2_h"], s["h_pows_inv"])
        if case["proof"] is None:
            with pytest.raises(hip.PlonkHipError):
                pr.prove(**_circuit(case), chal=case["chal"], rand=case["rand"])
        else:
            assert pr.prove(**_circuit(case), chal=case["chal"], rand=case["rand"]).hex() == case["proof"]


def _synthetic(n, seed, srs_len):
    """13 random 'interpolated' polynomials of length n, Z_H = x^n - 1, random SRS."""
    return gen.prove_instance(n, seed, srs_len)


@pytest.mark.parametrize("n,seed,z", [(256, 61, 0), (256, 62, 1), (4096, 63, 0), (16384, 61, 0), (16384, 64, 0),
                                      (16384, 65, None), (65536, 61, 0), (65536, 67, 16)])
def test_round5_divisions_vs_oracle(hip, oracle, n, seed, z):
    """Round 5's numerators and divisions by x - z, x - z omega: the one-launch forms -- the
    chunk aggregates from round 4's evaluation rows (PROVE_EVAL_AGG = 1, the default:
    lincomb_agg_divide_kernel, with the early commitments in its grid, in round 4's, or in neither)
    and the look-back form (PROVE_FUSE_DIV = 1, lincomb_divide_kernel: chunks in reverse block
    order, each waiting for the later chunks' aggregates) -- and the two-launch form give the
    oracle's proof, from 1 to ~32 chunks per division.  z = 0 is the shift q[j] = num[j + 1], which
    crosses lanes, waves and chunks (src/poly.h:124-177 with divisor x - 0)."""
    polys, chal, rnd, zh, pts = _synthetic(n, seed, 2 * n + 8)
    chal = list(chal)
    if z is not None:
        chal[3] = z
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    try:
        want = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes()).rounds(polys, chal, rnd, strict=False)
    except ProveError:   # (16384, 64, 0): t(x) too short for its slices -- the reference exits there too
        want = None
    for fuse, agg, early in ((1, 0, 1), (0, 1, 1), (0, 0, 1), (0, 1, 2), (0, 1, 0), (1, 1, 1), (0, 1, 1)):
        with hip.options(PROVE_FUSE_DIV=fuse, PROVE_EVAL_AGG=agg, PROVE_EARLY_COMMITS=early):
            if want is None:
                with pytest.raises(hip.PlonkHipError):
                    pr.rounds_dev(dev, chal, rnd, strict=False)
            else:
                assert pr.rounds_dev(dev, chal, rnd, strict=False).hex() == want.hex(), (fuse, agg, early)


@pytest.mark.parametrize("n,seed", [(37, 71), (4096, 72), (20000, 73)])
def test_commitments_srs_log_form(hip, oracle, n, seed):
    """The 9 commitments from the SRS in log form (PROVE_SRS_LOGS = 1: srs_log_kernel once at
    create; per proof commit_pack_kernel -- commitments, trimmed lengths and packing in one
    launch, with or without the 7 commitments that do not wait for round 5 running inside its scan
    launch -- or msm_log_kernel + trim_pack_kernel; committed lengths n + 2 .. n + 3, so 16-point
    groups plus a ragged tail) and from the G1 form give the oracle's proof, and the strict
    rejection (its status words) is the same in every form."""
    polys, chal, rnd, zh, pts = _synthetic(n, seed, 2 * n + 8)
    want = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes()).rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    for logs, fuse, early in ((1, 1, 1), (1, 1, 0), (1, 1, 2), (1, 0, 1), (0, 1, 1), (1, 1, 1)):
        with hip.options(PROVE_SRS_LOGS=logs, PROVE_PACK_FUSE=fuse, PROVE_EARLY_COMMITS=early):
            assert pr.rounds_dev(dev, chal, rnd, strict=False).hex() == want.hex(), (logs, fuse, early)
            with pytest.raises(hip.PlonkHipError, match="remainder"):
                pr.rounds_dev(dev, chal, rnd, strict=True)


def test_commitments_irregular_srs(hip, oracle):
    """An SRS with non-canonical encodings (an off-curve point, a coordinate >= 101): the log-form
    conversion flags it at create and the commitments take the exact serial folds of the raw
    bytes (src/srs.h:59-66 through src/g1.h's formulas), whatever PROVE_SRS_LOGS says."""
    n = 256
    polys, chal, rnd, zh, pts = _synthetic(n, 74, 2 * n + 8)
    pts = pts.copy()
    pts.reshape(-1)[3 * 5:3 * 5 + 3] = [7, 7, 0]       # off the curve y^2 = x^3 + 3
    pts.reshape(-1)[3 * 40:3 * 40 + 3] = [120, 3, 0]   # x >= 101
    want = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes()).rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    for logs in (1, 0):
        with hip.options(PROVE_SRS_LOGS=logs):
            assert pr.rounds_dev(dev, chal, rnd, strict=False).hex() == want.hex(), logs


@pytest.mark.parametrize("n,seed", [(8, 1), (37, 2), (256, 3), (1000, 4), (3000, 5), (2100, 6), (5000, 7)])
def test_rounds_shape_vs_oracle(hip, oracle, n, seed):
    """(n = 2100 and 5000: t_2 (4n + 6 coefficients) and (a b) q_m (3n + 2) need different
    transform sizes there, so they must not form one sum group -- ADVICE r3.)"""
    srs_len = 2 * n + 8
    polys, chal, rnd, zh, pts = _synthetic(n, seed, srs_len)
    ref = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes())
    want = ref.rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    got = pr.rounds_dev(dev, chal, rnd, strict=False)
    assert got.hex() == want.hex()
    # strict mode: synthetic numerators are not divisible by Z_H -- the reference exits
    with pytest.raises(hip.PlonkHipError):
        pr.rounds_dev(dev, chal, rnd, strict=True)
    with pytest.raises(ProveError):
        ref.rounds(polys, chal, rnd, strict=True)


def test_rounds_unaligned_inputs(hip, oracle):
    """Polynomials at odd device addresses: the rounds 1-3 preparation falls back from the fused
    16-byte kernel (prep_kernel) to the blinding poly_muls + lincombs; same bytes as the oracle."""
    n = 1000
    polys, chal, rnd, zh, pts = _synthetic(n, 4, 2 * n + 8)   # the n = 1000 case above (no reference exit)
    ref = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes())
    want = ref.rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    backing = [torch.zeros(n + 16, dtype=torch.uint8, device="cuda") for _ in polys]
    dev = []
    for b, p in zip(backing, polys):
        b[3:3 + n] = torch.from_numpy(p).to("cuda")
        dev.append(b[3:3 + n])
    assert all(t.data_ptr() % 16 == 3 for t in dev)
    assert pr.rounds_dev(dev, chal, rnd, strict=False).hex() == want.hex()
    aligned = [torch.from_numpy(p).to("cuda") for p in polys]
    assert pr.rounds_dev(aligned, chal, rnd, strict=False).hex() == want.hex()


def test_rounds_general_divisor(hip, oracle):
    """Z_H that is not x^m + c (H not a subgroup, e.g. n = 3): general long division path."""
    n = 3
    srs_len = 16
    polys, chal, rnd, _, pts = _synthetic(n, 11, srs_len)
    zh = np.frombuffer(oracle.poly_mul(oracle.poly_mul([16, 1], [13, 1]), [1, 1]), np.uint8)  # (x-1)(x-4)(x-16)
    ref = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes())
    want = ref.rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    got = pr.rounds_dev([torch.from_numpy(p).to("cuda") for p in polys], chal, rnd)
    assert got.hex() == want.hex()


def test_rounds_srs_too_short(hip, oracle):
    n = 64
    polys, chal, rnd, zh, pts = _synthetic(n, 21, n + 3)   # w_z(x) needs ~2n points
    ref = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes())
    with pytest.raises(ProveError):
        ref.rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    with pytest.raises(hip.PlonkHipError) as e:
        pr.rounds_dev([torch.from_numpy(p).to("cuda") for p in polys], chal, rnd)
    assert e.value.code == hip.PLK_ERR_RANGE


def test_rounds_deterministic_large(hip):
    """n = 2^16 prove-shaped run twice: identical bytes (no races in the pipeline)."""
    n = 1 << 16
    polys, chal, rnd, zh, pts = _synthetic(n, 31, 2 * n + 8)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    a = pr.rounds_dev(dev, chal, rnd)
    b = pr.rounds_dev(dev, chal, rnd)
    assert a == b and len(a) == 34


_BIG = {}


def _big_case(oracle):
    """n = 2^16 prove-shaped instance and its CPU answer (computed once per session)."""
    if not _BIG:
        n = 1 << 16
        polys, chal, rnd, zh, pts = _synthetic(n, 41, 2 * n + 8)
        ref = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes())
        _BIG.update(n=n, polys=polys, chal=chal, rnd=rnd, zh=zh, pts=pts,
                    want=ref.rounds(polys, chal, rnd, strict=False))
    return _BIG


def test_rounds_2_16_vs_oracle(hip, oracle):
    """n = 2^16: the batched round-3 products (2^17..2^19 transforms) against the oracle."""
    c = _big_case(oracle)
    pr = hip.Prover(c["n"], c["zh"], c["pts"])
    got = pr.rounds_dev([torch.from_numpy(p).to("cuda") for p in c["polys"]], c["chal"], c["rnd"])
    assert got.hex() == c["want"].hex()


def test_rounds_2_20_vs_golden(hip):
    """Config C5 itself: n = 2^20 gates, the 34 proof bytes against the CPU oracle's answer
    (tests/golden/prove_2_20.json, made by tests/golden/make_prove_2_20.py -- 21 s of oracle
    time, so recorded once rather than recomputed here)."""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = _synthetic(n, g["seed"], g["srs_len"])
    pr = hip.Prover(n, zh, pts)
    got = pr.rounds_dev([torch.from_numpy(p).to("cuda") for p in polys], chal, rnd)
    assert got.hex() == g["proof"]


def test_profile_and_launch_count_2_20(hip):
    """The C5 line's measurement entry points: plk_prover_profile_dev gives the
    recorded proof bytes with its event times consistent (both product batches inside the launch
    sequence); plk_prover_launches counts the proof's kernels from a captured, never launched graph
    -- 12 at 2^20 gates plain, 11 preprocessed (no shared-operand pass; DESIGN 4b,
    profiles/r05_prove_2^20_*breakdown.txt) -- without changing what the next call
    computes; the launch plan holds the 7 NTT pass launches of the two batches, all over F29."""
    from plonkhip import roofline as RL
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = _synthetic(n, g["seed"], g["srs_len"])
    d = [torch.from_numpy(p).to("cuda") for p in polys]
    pr = hip.Prover(n, zh, pts)
    for pre in (False, True):
        if pre:
            pr.preprocess(d)
        assert pr.launches(d, chal, rnd, preprocessed=pre) == (11 if pre else 12, 0)
        assert pr.rounds_dev(d, chal, rnd, preprocessed=pre).hex() == g["proof"]
        hip.ntt_launch_log()
        with hip.options(NTT_LAUNCH_LOG=1):
            got, ms = pr.profile_dev(d, chal, rnd, preprocessed=pre)
        plan = hip.ntt_launch_log()
        assert got.hex() == g["proof"]
        assert 0 < ms["batch1_ms"] and 0 < ms["batch2_ms"] and ms["ntt_ms"] < ms["span_ms"] < 5.0, ms
        assert [r["field"] for r in plan] == [0] * len(plan)
        assert sorted(r["kind"] for r in plan) == ([0, 0, 1, 1, 2, 2] if pre else [0, 0, 1, 1, 2, 2, 3])
        tot = RL.plan_roofline(plan, RL.load_peaks(RL.PEAKS))
        assert tot["roof_s"] * 1e3 < ms["ntt_ms"]          # the roof is below the measured time
    assert pr.alg_bytes() > 9 * 4 * n


def test_profile_and_launches_small_vs_rounds(hip):
    """at n = 4096 the profiled proof and the counted capture leave rounds_dev's answer unchanged,
    call after call (the capture restores the completion-word sequence it advanced)"""
    polys, chal, rnd, zh, pts = _synthetic(4096, 9, 2 * 4096 + 8)
    d = [torch.from_numpy(p).to("cuda") for p in polys]
    pr = hip.Prover(4096, zh, pts)
    want = pr.rounds_dev(d, chal, rnd)
    k, _ = pr.launches(d, chal, rnd)
    assert 8 <= k <= 20
    assert pr.rounds_dev(d, chal, rnd) == want
    assert pr.profile_dev(d, chal, rnd)[0] == want
    assert pr.rounds_dev(d, chal, rnd) == want
    with hip.options(PROVE_GRAPH=1):
        assert pr.rounds_dev(d, chal, rnd) == want and pr.rounds_dev(d, chal, rnd) == want


@pytest.mark.parametrize("n,seed", [(256, 3), (3000, 5), (5000, 7), (1 << 16, 41)])
def test_derive_t2a_modes_vs_oracle(hip, oracle, n, seed):
    """Round 3's A2 B2 three ways (PLK_OPT_PROVE_DERIVE_T2A): its own product (0), t2a_kernel (1),
    and inside the t_2 product's first forward pass (2, 2^13-tile products only: here t_2 runs on
    2^12 tiles, so mode 2 takes mode 1's kernel -- the derived pass itself is checked against the
    oracle by test_rounds_2_16_tiles13_vs_oracle, where every transform uses 2^13 tiles, and
    against the golden at 2^20)."""
    if n == 1 << 16:
        c = _big_case(oracle)
        polys, chal, rnd, zh, pts, want = c["polys"], c["chal"], c["rnd"], c["zh"], c["pts"], c["want"]
    else:
        polys, chal, rnd, zh, pts = _synthetic(n, seed, 2 * n + 8)
        want = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes()).rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    for mode in (0, 1, 2):
        with hip.options(PROVE_DERIVE_T2A=mode):
            assert pr.rounds_dev(dev, chal, rnd, strict=False).hex() == want.hex(), mode


def test_derive_t2a_2_20_vs_golden(hip):
    """Config C5 with A2 B2 computed by t2a_kernel and inside the t_2 product's first forward pass."""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = _synthetic(n, g["seed"], g["srs_len"])
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    for mode in (1, 2):
        with hip.options(PROVE_DERIVE_T2A=mode):
            assert pr.rounds_dev(dev, chal, rnd).hex() == g["proof"], mode
            pr.preprocess(dev)
            assert pr.rounds_dev(dev, chal, rnd, preprocessed=True).hex() == g["proof"], mode
            pr.preprocess(None)


@pytest.mark.parametrize("n,seed", [(3000, 5), (1 << 16, 41)])
def test_graph_replay_vs_direct(hip, n, seed):
    """PLK_OPT_PROVE_GRAPH: the first call captures the proof's launches, later calls replay them
    with the scalar file and the completion word set per call -- the same bytes as direct launches
    for two challenge / blinding sets in turn, plain and preprocessed (a recapture: the fixed
    transforms changed), after an input moved (recapture), and again with the graph off."""
    polys, chal, rnd, zh, pts = _synthetic(n, seed, 2 * n + 8)
    sets = [(list(chal), list(rnd)), (list(chal[1:]) + [chal[0]], list(rnd[::-1]))]
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    want = [pr.rounds_dev(dev, c, r) for c, r in sets]
    assert want[0] != want[1]
    with hip.options(PROVE_GRAPH=1):
        for _ in range(3):
            for (c, r), w in zip(sets, want):
                assert pr.rounds_dev(dev, c, r).hex() == w.hex()
        pr.preprocess(dev)
        for _ in range(2):
            for (c, r), w in zip(sets, want):
                assert pr.rounds_dev(dev, c, r, preprocessed=True).hex() == w.hex()
        moved = list(dev)
        moved[5] = dev[5].clone()
        for (c, r), w in zip(sets, want):
            assert pr.rounds_dev(moved, c, r, preprocessed=True).hex() == w.hex()
        pr.preprocess(None)
        assert pr.rounds_dev(dev, *sets[1]).hex() == want[1].hex()
    # the fused look-back division changes its scan epoch per call: such calls run direct launches
    with hip.options(PROVE_GRAPH=1, PROVE_FUSE_DIV=1):
        for _ in range(2):
            for (c, r), w in zip(sets, want):
                assert pr.rounds_dev(dev, c, r).hex() == w.hex()
    assert pr.rounds_dev(dev, *sets[0]).hex() == want[0].hex()


def test_graph_replay_2_20_vs_golden(hip):
    """Config C5 through the captured graph: capture, then replays, all the golden bytes."""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = _synthetic(n, g["seed"], g["srs_len"])
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    with hip.options(PROVE_GRAPH=1):
        for _ in range(3):
            assert pr.rounds_dev(dev, chal, rnd).hex() == g["proof"]


_TILE13_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = sys.argv[1:2]
import plonkhip as hip
hip.set_option("NTT_T13_MIN_K", 13)   # shapes the column tables: before plk_init
hip.init(0)
d = np.load(sys.argv[2])
n = int(d["n"])
polys = [torch.from_numpy(d["p%d" % i]).to("cuda") for i in range(13)]
pr = hip.Prover(n, d["zh"], d["pts"])
print(pr.rounds_dev(polys, [int(x) for x in d["chal"]], [int(x) for x in d["rnd"]]).hex())
"""


def test_rounds_2_16_tiles13_vs_oracle(hip, oracle, tmp_path):
    """Same instance with every transform on the 2^13-element tile engine (PLK_OPT_NTT_T13_MIN_K
    = 13, set before plk_init: a child process), so the batched prover runs the tile size
    that 2^21..2^23 products use at n = 2^20."""
    import os
    import subprocess
    import sys
    c = _big_case(oracle)
    f = tmp_path / "case.npz"
    np.savez(f, n=c["n"], zh=c["zh"], pts=c["pts"], chal=np.array(c["chal"]), rnd=np.array(c["rnd"]),
             **{"p%d" % i: p for i, p in enumerate(c["polys"])})
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plonk.c_amd")
    r = subprocess.run([sys.executable, "-c", _TILE13_SCRIPT, pkg, str(f)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == c["want"].hex()


def test_rounds_preprocessed_vs_golden(hip):
    """Config C5 with a preprocessed circuit (plk_prover_preprocess: the six fixed polynomials'
    round-3 transforms computed once): the same proof bytes as the golden, repeatedly, and the
    plain path unchanged beside it; a fixed polynomial moved to another address is transformed
    in the call again (its stale transform is not used)."""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = _synthetic(n, g["seed"], g["srs_len"])
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    pr.preprocess(dev)
    for _ in range(2):
        assert pr.rounds_dev(dev, chal, rnd, preprocessed=True).hex() == g["proof"]
    assert pr.rounds_dev(dev, chal, rnd).hex() == g["proof"]
    moved = list(dev)
    moved[5] = dev[5].clone()                       # q_l at a new address
    assert pr.rounds_dev(moved, chal, rnd, preprocessed=True).hex() == g["proof"]
    pr.preprocess(None)
    assert pr.rounds_dev(dev, chal, rnd, preprocessed=True).hex() == g["proof"]


@pytest.mark.parametrize("n,seed", [(1 << 16, 41), (1 << 12, 7), (64, 3)])
def test_rounds_preprocessed_vs_plain(hip, n, seed):
    """Preprocessed and plain provers agree at sizes whose round-3 products run at 2^13..2^19
    transforms (12- and 13-bit tiles) and at a size with no transform-engine product at all."""
    polys, chal, rnd, zh, pts = _synthetic(n, seed, 2 * n + 8)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    want = pr.rounds_dev(dev, chal, rnd)
    pr.preprocess(dev)
    assert pr.rounds_dev(dev, chal, rnd, preprocessed=True).hex() == want.hex()


def test_rounds_challenge_forms_agree(hip):
    """rounds_dev normalises chal / rand like prove(): int64 numpy arrays, lists and bytes give
    the same proof (a raw byte copy of an int64 array would put zeros in 4 of 5 challenges); a
    wrong count is an error, not silent padding."""
    n = 1 << 10
    polys, chal, rnd, zh, pts = _synthetic(n, 5, 2 * n + 8)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    want = pr.rounds_dev(dev, list(chal), list(rnd))
    assert pr.rounds_dev(dev, np.array(list(chal), np.int64), np.array(list(rnd), np.int64)) == want
    assert pr.rounds_dev(dev, bytes(list(chal)), bytes(list(rnd))) == want
    with pytest.raises(ValueError):
        pr.rounds_dev(dev, list(chal)[:4], list(rnd))
    with pytest.raises(ValueError):
        pr.rounds_dev(dev, list(chal), list(rnd) + [1])


def test_preprocessed_tensors_held_and_overwrite_needs_preprocess(hip):
    """The preprocessed transforms are bound to device addresses: the Prover keeps the tensors it
    was given alive (their addresses cannot be handed to another circuit), and new bytes written
    in place at those addresses take effect after preprocess() is called again (the contract in
    include/plonkhip.h) -- equal to the plain proof of the new bytes."""
    n = 1 << 12
    polys, chal, rnd, zh, pts = _synthetic(n, 9, 2 * n + 8)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    pr.preprocess(dev)
    assert pr._fixed is not None and all(a is b for a, b in zip(pr._fixed, dev))
    polys2, _, _, _, _ = _synthetic(n, 10, 2 * n + 8)
    for i in (3, 4, 5, 6, 10, 12):                     # the fixed circuit polynomials, in place
        dev[i].copy_(torch.from_numpy(polys2[i]).to("cuda"))
    want = pr.rounds_dev(dev, chal, rnd)                # plain: reads the new bytes
    pr.preprocess(dev)
    assert pr.rounds_dev(dev, chal, rnd, preprocessed=True) == want
    pr.preprocess(None)
    assert pr._fixed is None


# every switch that changes how a 2^20 proof is computed, one at a time away from its default
_SWEEP = [("NTT_F29", 0), ("NTT_SHARE", 0), ("NTT_SHARED_FIX", 0), ("NTT_SHARED_FIX", 2), ("NTT_CENTER_BLOCKS", 768),
          ("NTT_CENTER_SUM", 0), ("NTT_TABLE_SHARE", 0), ("PROVE_DERIVE_T2A", 0), ("PROVE_DERIVE_T2A", 1),
          ("PROVE_FUSE_DIV", 1), ("PROVE_SRS_LOGS", 0), ("PROVE_PACK_FUSE", 0), ("PROVE_EARLY_COMMITS", 0),
          ("PROVE_EARLY_COMMITS", 2), ("PROVE_EVAL_AGG", 0), ("PROVE_GRAPH", 1), ("PROVE_SYNC", 1)]


def test_option_sweep_2_20_vs_golden(hip):
    """Config C5 with each computation switch (PLK_OPT_*) moved off its default in turn -- BabyBear
    instead of F29, no shared operands, the shared-operand pass off / forced, another centre grid,
    no centre sum groups, per-array column reads, A2 B2 as a product or its own kernel, the fused
    look-back division, G1-form commitments, unfused packing, the early commitments elsewhere, the
    two-launch division, graph replay, stream-synchronised completion -- plain and preprocessed:
    the golden bytes every time (round 5 found a wrong-result bug behind a non-default option)."""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = _synthetic(n, g["seed"], g["srs_len"])
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    for opt, val in _SWEEP:
        with hip.options(**{opt: val}):
            assert pr.rounds_dev(dev, chal, rnd).hex() == g["proof"], (opt, val)
    pr.preprocess(dev)
    for opt, val in _SWEEP:
        with hip.options(**{opt: val}):
            assert pr.rounds_dev(dev, chal, rnd, preprocessed=True).hex() == g["proof"], (opt, val, "pre")
