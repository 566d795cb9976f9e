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


# ---- the distinct-device input path, executed on one GPU
HELPER_IN = (0, 1, 2, 8, 9, 10, 11)      # f_a f_b f_c s_sigma_1..3 acc_x: what a helper's chains read


@pytest.fixture
def helper_copy(hip):
    """PLK_OPT_PROVE_HELPER_COPY: helpers on the proving device take the distinct-device input
    branch of rounds_split (inputs copied into their own rows, the other six entries pointed at a
    poison row of 0x05 bytes) -- the branch an 8-GPU node runs"""
    hip.set_option("PROVE_HELPER_COPY", 1)
    yield
    hip.set_option("PROVE_HELPER_COPY", 0)


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("n,seed", [(1 << 12, 7), (5000, 7), (64, 3)])
def test_helper_input_copy_branch(hip, devlist, helper_copy, k, n, seed):
    devlist([0] * (1 + k))
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    dev = _dev(polys)
    single = hip.Prover(n, zh, pts)
    want = single.rounds_dev(dev, chal, rnd)
    pr = hip.Prover(n, zh, pts)
    pr.attach_helpers(k)
    for _ in range(2):
        assert pr.rounds_dev(dev, chal, rnd).hex() == want.hex()
    # new inputs in the same device buffers: the copies must carry them (not the first call's rows)
    polys2, _, _, _, _ = gen.prove_instance(n, seed + 1, 2 * n + 8)
    for d, p in zip(dev, polys2):
        d.copy_(torch.from_numpy(p))
    assert pr.rounds_dev(dev, chal, rnd).hex() == single.rounds_dev(dev, chal, rnd).hex()
    pr.close()
    single.close()


@pytest.mark.parametrize("k", [1, 2])
def test_helper_input_copy_branch_2_20(hip, devlist, helper_copy, k):
    """config C5 through the copy branch at 2 and 3 'devices': the recorded answer"""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    devlist([0] * (1 + k))
    polys, chal, rnd, zh, pts = gen.prove_instance(n, g["seed"], g["srs_len"])
    pr = hip.Prover(n, zh, pts)
    pr.attach_helpers(k)
    assert pr.rounds_dev(_dev(polys), chal, rnd).hex() == g["proof"]
    pr.close()


@pytest.mark.parametrize("k", [1, 2])
def test_multi_dev_helpers_read_only_their_inputs(hip, devlist, k):
    """plk_prover_rounds_multi_dev with every helper set's six entries outside HELPER_IN pointed
    at poison (0x05 bytes): the proof is unchanged, i.e. a helper reads nothing else (the claim
    rounds_split's copies rest on).  Control: poisoning one HELPER_IN entry changes the proof."""
    n = 1 << 12
    devlist([0] * (1 + k))
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 9, 2 * n + 8)
    dev = _dev(polys)
    poison = torch.full((n + 64,), 5, dtype=torch.uint8, device="cuda")
    pr = hip.Prover(n, zh, pts)
    want = pr.rounds_dev(dev, chal, rnd)
    pr.attach_helpers(k)
    hsets = [[d if i in HELPER_IN else poison for i, d in enumerate(dev)] for _ in range(k)]
    assert pr.rounds_multi_dev([dev] + hsets, chal, rnd).hex() == want.hex()
    bad = [list(s) for s in hsets]
    bad[-1][HELPER_IN[0]] = poison
    assert pr.rounds_multi_dev([dev] + bad, chal, rnd).hex() != want.hex()
    pr.close()


_DROP_CHILD = r"""
import sys
sys.path[:0] = sys.argv[1:3]
import torch, gen, plonkhip as hip
hip.init(0)
hip.set_option("PROVE_HELPER_COPY", 1)
n = 1 << 12
polys, chal, rnd, zh, pts = gen.prove_instance(n, 7, 2 * n + 8)
dev = [torch.from_numpy(p).to("cuda") for p in polys]
single = hip.Prover(n, zh, pts)
want = single.rounds_dev(dev, chal, rnd).hex()
for k in (1, 2):
    hip.init_devices([0] * (1 + k))
    pr = hip.Prover(n, zh, pts)
    pr.attach_helpers(k)
    try:
        got = pr.rounds_dev(dev, chal, rnd).hex()
    except hip.PlonkHipError as e:   # (wrong chain bytes can make the proof fail its checks)
        got = "error-%d" % e.code
    print(k, got, want)
    pr.close()
hip.init_devices([0])
"""


def test_skipped_input_copy_is_caught():
    """a build whose copy branch skips one of the seven input copies (f_a; PLK_DIAG_DROP_HANDOFF = 4)
    gives wrong proof bytes at 2 and 3 'devices': the helper then reads its poison row, so the test
    above would catch a missing copy.  The real build, in the same child form, is exact."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = [os.path.join(root, "plonk.c_amd"), os.path.join(root, "tests", "golden")]

    def run(lib):
        r = subprocess.run([sys.executable, "-c", _DROP_CHILD, *paths], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, PLK_LIB=lib))
        assert r.returncode == 0, r.stderr[-2000:]
        return [l.split() for l in r.stdout.splitlines() if l[:1] in "12"]

    lib = os.path.join(root, "plonk.c_amd", "build", "diag", "libplonkhip_drop4.so")
    assert os.path.exists(lib), "diagnostic build missing: make -C plonk.c_amd diag (__graft_entry__.build does)"
    rows = run(lib)
    assert len(rows) == 2
    for k, got, want in rows:
        assert got != want, "skipped input copy not caught with %s helper(s)" % k
    rows = run(os.path.join(root, "plonk.c_amd", "libplonkhip.so"))
    assert len(rows) == 2 and all(got == want for _, got, want in rows)


def test_prover_calls_from_another_thread(hip):
    """every prover entry point runs on the prover's own device whatever the calling thread's
    current device (tables are looked up by the current device): calls from a fresh
    thread -- and, with two or more GPUs, from a thread current on another device -- give the
    same proof"""
    import threading
    n = 1 << 12
    polys, chal, rnd, zh, pts = gen.prove_instance(n, 11, 2 * n + 8)
    dev = _dev(polys)
    pr = hip.Prover(n, zh, pts)
    want = pr.rounds_dev(dev, chal, rnd)
    other = 1 if torch.cuda.device_count() > 1 else 0
    out = {}

    def worker():
        try:
            torch.cuda.set_device(other)
            out["plain"] = pr.rounds_dev(dev, chal, rnd)
            pr.preprocess(dev)
            out["pre"] = pr.rounds_dev(dev, chal, rnd, preprocessed=True)
            out["dev_after"] = torch.cuda.current_device()
        except Exception as e:   # noqa: BLE001 -- reported below
            out["err"] = repr(e)

    t = threading.Thread(target=worker)
    t.start()
    t.join(120)
    assert "err" not in out, out.get("err")
    assert out["plain"] == want and out["pre"] == want
    assert out["dev_after"] == other              # the caller's device is restored
    pr.close()
