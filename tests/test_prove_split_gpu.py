"""Strong-scaled proof entry points (plk_prover_chains_dev / plk_prover_rounds_ext_dev, SURVEY §8e:
round 3's product chains t_2 = (A2 B2)(C2 z) and t_3 = (A3 B3)(C3 z(omega x)),
src/plonk.h:432-434, 471-473, computed by another prover from the same inputs).  Rehearsed on one
GPU: the helper provers run on their own streams of the same device, and the proving call reads
their products after an event on the helper's stream -- the same hand-off the multi-GPU bench leg
makes over RCCL.  The proof bytes must equal the single-prover proof and, at n = 2^20, the
recorded answer of the CPU restatement (tests/golden/prove_2_20.json)."""
import pytest
import torch

import gen
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _split_proof(hip, n, polys, chal, rnd, zh, pts, which, helpers=1, preprocessed=False, side_stream=True):
    """which: chain mask the helpers compute; helpers = 1 (one prover for every chain in `which`)
    or 2 (one prover per chain)"""
    main = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    if preprocessed:
        main.preprocess(dev)
    t2 = torch.zeros(main.chain_bytes(hip.PLK_CHAIN_T2), dtype=torch.uint8, device="cuda")
    t3 = torch.zeros(main.chain_bytes(hip.PLK_CHAIN_T3), dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream() if side_stream else torch.cuda.current_stream()   # (the default: the null stream)
    masks = [which] if helpers == 1 else [m for m in (hip.PLK_CHAIN_T2, hip.PLK_CHAIN_T3) if which & m]
    hs = [hip.Prover(n, zh, pts) for _ in masks]
    for h, m in zip(hs, masks):
        h.chains_dev(dev, chal, rnd, m, t2 if m & hip.PLK_CHAIN_T2 else None, t3 if m & hip.PLK_CHAIN_T3 else None,
                     done=st)
    got = main.rounds_ext_dev(dev, chal, rnd, which, t2 if which & hip.PLK_CHAIN_T2 else None,
                              t3 if which & hip.PLK_CHAIN_T3 else None, ready=st, preprocessed=preprocessed)
    want = main.rounds_dev(dev, chal, rnd)
    for h in hs:
        h.close()
    main.close()
    return got, want


@pytest.mark.parametrize("which,helpers,side", [(1, 1, True), (2, 1, True), (3, 1, True), (3, 2, True), (3, 1, False)])
def test_split_matches_single_prover(hip, which, helpers, side):
    """side = False: the hand-off through torch's default (null) stream, as the bench leg does"""
    n = 1 << 16
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 41, 2 * n + 8)
    got, want = _split_proof(hip, n, polys, chal, rnd, zh, pts, which, helpers, side_stream=side)
    assert got.hex() == want.hex()


@pytest.mark.parametrize("n,seed", [(1 << 12, 7), (64, 3)])
def test_split_small_sizes(hip, n, seed):
    """12-bit tiles and products below the transform engine (direct / small kernels)"""
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    got, want = _split_proof(hip, n, polys, chal, rnd, zh, pts, 3, 2)
    assert got.hex() == want.hex()


def test_split_2_20_vs_golden(hip):
    """Config C5: both chains on helper provers, plain and preprocessed main prover"""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = gen.prove_instance(n, g["seed"], g["srs_len"])
    got, want = _split_proof(hip, n, polys, chal, rnd, zh, pts, 3, 2)
    assert got.hex() == want.hex() == g["proof"]
    got, _ = _split_proof(hip, n, polys, chal, rnd, zh, pts, 3, 1, preprocessed=True)
    assert got.hex() == g["proof"]


def test_split_argument_errors(hip):
    n = 1 << 10
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 5, 2 * n + 8)
    pr = hip.Prover(n, zh, pts)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    assert pr.chain_bytes(hip.PLK_CHAIN_T2) > 4 * n and pr.chain_bytes(hip.PLK_CHAIN_T3) > 4 * n   # (t_2, t_3: ~4n + 6 coefficients)
    assert pr.chain_bytes(4) == 0
    with pytest.raises(hip.PlonkHipError):
        pr.chains_dev(dev, chal, rnd, hip.PLK_CHAIN_T2, None, None)        # no buffer for the chain
    with pytest.raises(hip.PlonkHipError):
        pr.rounds_ext_dev(dev, chal, rnd, 4)                               # bad mask
    buf = torch.zeros(pr.chain_bytes(hip.PLK_CHAIN_T3) + 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(hip.PlonkHipError):
        pr.rounds_ext_dev(dev, chal, rnd, hip.PLK_CHAIN_T3, None, buf[1:])  # misaligned
    pr.close()


def _oracle_want(oracle, n, polys, chal, rnd, zh, pts):
    from prove_ref import Prover as RefProver
    return RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes()).rounds(polys, chal, rnd, strict=False)


def _split_on(hip, n, dev, chal, rnd, zh, pts, which=3, strict=False):
    """helpers on the null stream, the proving prover reading after it"""
    main, helper = hip.Prover(n, zh, pts), hip.Prover(n, zh, pts)
    t2 = torch.zeros(main.chain_bytes(hip.PLK_CHAIN_T2), dtype=torch.uint8, device="cuda")
    t3 = torch.zeros(main.chain_bytes(hip.PLK_CHAIN_T3), dtype=torch.uint8, device="cuda")
    try:
        helper.chains_dev(dev, chal, rnd, which, t2, t3)
        return main.rounds_ext_dev(dev, chal, rnd, which, t2, t3, strict=strict)
    finally:
        helper.close()
        main.close()


@pytest.mark.parametrize("n,seed", [(8, 1), (1000, 4), (3000, 5)])
def test_split_vs_oracle(hip, oracle, n, seed):
    """the split proof against the CPU restatement (oracle/prove_ref.py) directly"""
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    assert _split_on(hip, n, dev, chal, rnd, zh, pts).hex() == _oracle_want(oracle, n, polys, chal, rnd, zh, pts).hex()


@pytest.mark.parametrize("n,seed", [(2100, 6), (5000, 7)])
def test_split_vs_oracle_group_sizes(hip, oracle, n, seed):
    """sizes where t_2 and (a b) q_m land on different transform sizes (no sum group): rank 0
    keeping t_2 (the N = 2 split, only t_3 received) and receiving both"""
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    want = _oracle_want(oracle, n, polys, chal, rnd, zh, pts).hex()
    for which in (hip.PLK_CHAIN_T3, hip.PLK_CHAIN_T2 | hip.PLK_CHAIN_T3):
        assert _split_on(hip, n, dev, chal, rnd, zh, pts, which).hex() == want


def test_split_unaligned_inputs(hip, oracle):
    """odd device addresses: both sides fall back from prep_kernel to the poly_mul + lincomb
    preparation; the numerator then runs as a lincomb + division instead of numdiv_kernel"""
    n = 1000
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 4, 2 * n + 8)
    backing = [torch.zeros(n + 16, dtype=torch.uint8, device="cuda") for _ in polys]
    dev = []
    for b, p in zip(backing, polys):
        b[3:3 + n] = torch.from_numpy(p).to("cuda")
        dev.append(b[3:3 + n])
    for which in (1, 2, 3):
        assert _split_on(hip, n, dev, chal, rnd, zh, pts, which).hex() == \
            _oracle_want(oracle, n, polys, chal, rnd, zh, pts).hex()


def test_split_general_divisor(hip, oracle):
    """Z_H not of the form x^m + c (the general long division after the received chains)"""
    import numpy as np
    n = 3
    polys, chal, rnd, _, pts = gen.prove_instance(n, 11, 16)
    zh = np.frombuffer(oracle.poly_mul(oracle.poly_mul([16, 1], [13, 1]), [1, 1]), np.uint8)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    assert _split_on(hip, n, dev, chal, rnd, zh, pts).hex() == _oracle_want(oracle, n, polys, chal, rnd, zh, pts).hex()


def test_split_reference_exits(hip):
    """strict: the synthetic numerator is not divisible by Z_H (the reference exits) -- an error
    through the split path too; an SRS too short for w_z(x) -> PLK_ERR_RANGE"""
    n = 64
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 21, 2 * n + 8)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    with pytest.raises(hip.PlonkHipError):
        _split_on(hip, n, dev, chal, rnd, zh, pts, strict=True)
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 21, n + 3)
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    with pytest.raises(hip.PlonkHipError) as e:
        _split_on(hip, n, dev, chal, rnd, zh, pts)
    assert e.value.code == hip.PLK_ERR_RANGE
