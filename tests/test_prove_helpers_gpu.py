"""One proof over several GPUs driven from C (plk_prover_attach_helpers): helper
provers on entries 1..k of the plk_init_devices list compute round 3's t_2 / t_3 chains
(src/plonk.h:432-434, 471-473) on their own streams, their products reach the proving device by
hipMemcpyPeerAsync behind an event, and the proving stream waits for those events only before its
numerator.  Rehearsed on one GPU with lists repeating device 0 ([0, 0]: t_3 on a helper; [0, 0, 0]:
t_2 and t_3), as the sharded MSM is: the proof bytes equal the single-prover proof, the CPU
restatement's answer (oracle/prove_ref.py) and, at 2^20 gates, the recorded answer
tests/golden/prove_2_20.json.  Distinct devices: unmeasured here (one-GPU boxes)."""
import pytest
import torch

import gen
from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture
def devlist(hip):
    """sets the plk_init_devices list for a test, back to one device after it"""
    def use(ids):
        hip.init_devices(ids)
    yield use
    hip.init_devices([0])


def _dev(polys):
    return [torch.from_numpy(p).to("cuda") for p in polys]


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("n,seed", [(1 << 16, 41), (1 << 12, 7), (5000, 7), (64, 3), (8, 1)])
def test_helpers_match_single_prover(hip, devlist, k, n, seed):
    devlist([0] * (1 + k))
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    dev = _dev(polys)
    single = hip.Prover(n, zh, pts)
    want = single.rounds_dev(dev, chal, rnd)
    pr = hip.Prover(n, zh, pts)
    pr.attach_helpers(k)
    assert pr.helpers() == k
    for _ in range(2):                               # (buffers and events reused by the next proof)
        assert pr.rounds_dev(dev, chal, rnd).hex() == want.hex()
    assert pr.rounds_multi_dev([dev] * (1 + k), chal, rnd).hex() == want.hex()
    pr.attach_helpers(0)
    assert pr.helpers() == 0
    assert pr.rounds_dev(dev, chal, rnd).hex() == want.hex()
    pr.close()
    single.close()


@pytest.mark.parametrize("n,seed", [(1000, 4), (2100, 6)])
def test_helpers_vs_oracle(hip, oracle, devlist, n, seed):
    from prove_ref import Prover as RefProver
    devlist([0, 0, 0])
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    want = RefProver(oracle, pts.tobytes(), n, z_h=zh.tobytes()).rounds(polys, chal, rnd, strict=False)
    pr = hip.Prover(n, zh, pts)
    for k in (1, 2):
        pr.attach_helpers(k)
        assert pr.rounds_dev(_dev(polys), chal, rnd).hex() == want.hex()
    pr.close()


@pytest.mark.parametrize("k", [1, 2])
def test_helpers_2_20_vs_golden(hip, devlist, k):
    """config C5 through 2 and 3 'devices', plain and preprocessed proving prover"""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    devlist([0] * (1 + k))
    polys, chal, rnd, zh, pts = gen.prove_instance(n, g["seed"], g["srs_len"])
    dev = _dev(polys)
    pr = hip.Prover(n, zh, pts)
    pr.attach_helpers(k)
    assert pr.rounds_dev(dev, chal, rnd).hex() == g["proof"]
    pr.preprocess(dev)
    assert pr.rounds_dev(dev, chal, rnd, preprocessed=True).hex() == g["proof"]
    pr.close()


def test_helpers_circuit_proofs(hip, devlist):
    """plk_prover_prove (the circuit path: stage A on the proving device, the helpers' inputs
    taken after it) reproduces the reference's 4-gate proofs with helpers attached"""
    from test_prove_gpu import _circuit, _setup
    devlist([0, 0, 0])
    g = load_golden("prove.json")
    provers = {}
    for case in g["proofs"][:8]:
        key = (case["srs_n"], case["srs_mode"])
        if key not in provers:
            s = _setup(g, case)
            provers[key] = hip.Prover(4, s["z_h"], s["g1s"], s["h"], s["k1_h"], s["k2_h"], s["h_pows_inv"])
            provers[key].attach_helpers(2)
        got = provers[key].prove(**_circuit(case), chal=case["chal"], rand=case["rand"])
        assert got.hex() == case["proof"]
    for p in provers.values():
        p.close()


def test_attach_errors(hip, devlist):
    n = 1 << 10
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 5, 2 * n + 8)
    pr = hip.Prover(n, zh, pts)
    devlist([0])
    with pytest.raises(hip.PlonkHipError):
        pr.attach_helpers(1)                          # the list has no second entry
    devlist([0, 0])
    with pytest.raises(hip.PlonkHipError):
        pr.attach_helpers(2)
    with pytest.raises(hip.PlonkHipError):
        pr.attach_helpers(3)
    assert pr.helpers() == 0
    pr.attach_helpers(1)
    dev = _dev(polys)
    with pytest.raises(hip.PlonkHipError):
        pr.rounds_multi_dev([dev], chal, rnd)         # one input set for two devices
    pr.close()
