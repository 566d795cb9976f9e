"""The device (RCCL) branch of the strong-scaled proof, rehearsed on one GPU.

plonkhip.dist.split_proof_step(..., via_host=False) -- the branch bench.py's prove_split_component
takes over RCCL on a multi-GPU node -- driven through tests/nccl_standin.py, a torch.distributed
stand-in with RCCL's stream semantics (a send reads its tensor when the caller's current stream
gets there; a receive lands late on a side stream and wait() only makes the current stream wait).
The orderings under test:
  * helper: plk_prover_chains_dev(done=stream) makes `stream` wait for the chains, so the send
    (ordered behind `stream`) reads finished products;
  * rank 0: plk_prover_rounds_ext_dev(ready=stream) makes the prover's stream wait for everything
    on `stream` at the call -- the receive's wait() -- before its numerator reads the chains.
The real library gives the single-prover proof (and the recorded 2^20 answer); the diagnostic
builds with one ordering removed (plonk.c_amd/Makefile `diag`, PLK_DIAG_DROP_HANDOFF in prove.hip)
must give WRONG bytes through the same stand-in -- i.e. the test catches a missing ordering.
Reference: round 3's t_2 / t_3 chains, src/plonk.h:432-434, 471-473."""
import os
import subprocess
import sys

import pytest

import gen
from conftest import load_golden
from nccl_standin import split_proof

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,n,seed", [(2, 1 << 16, 41), (3, 1 << 16, 41), (3, 1 << 12, 7), (2, 5000, 7)])
def test_device_branch_matches_single_prover(hip, world, n, seed):
    polys, chal, rnd, zh, pts = gen.prove_instance(n, seed, 2 * n + 8)
    got, want = split_proof(hip, n, polys, chal, rnd, zh, pts, world)
    assert got is not None and got.hex() == want.hex()


def test_device_branch_2_20_vs_golden(hip):
    """config C5 at 3 ranks: the recorded answer of the CPU restatement"""
    g = load_golden("prove_2_20.json")
    n = g["n"]
    polys, chal, rnd, zh, pts = gen.prove_instance(n, g["seed"], g["srs_len"])
    got, want = split_proof(hip, n, polys, chal, rnd, zh, pts, 3)
    assert got.hex() == want.hex() == g["proof"]


_CHILD = r"""
import sys
sys.path[:0] = sys.argv[1:4]
import gen, plonkhip as hip
from nccl_standin import split_proof
hip.init(0)
n = 1 << 20   # (chains of ~0.15 ms: an unordered send copies long before they end)
polys, chal, rnd, zh, pts = gen.prove_instance(n, 51, 2 * n + 8)
want = None
for world in (2, 3):
    try:
        got, want = split_proof(hip, n, polys, chal, rnd, zh, pts, world)
        got = got.hex()
    except hip.PlonkHipError as e:   # (wrong chain bytes can also make the proof fail: t(x) too short)
        got = "error-%d" % e.code
    if want is None:
        pr = hip.Prover(n, zh, pts)
        import torch
        want = pr.rounds_dev([torch.from_numpy(p).to("cuda") for p in polys], chal, rnd)
        pr.close()
    print(world, got, want.hex())
"""


def _child(lib):
    env = dict(os.environ)
    env["PLK_LIB"] = lib
    # one hardware queue per stream (nccl_standin's docstring): streams sharing a queue run in
    # submission order, which would hide the race a missing ordering opens
    env["GPU_MAX_HW_QUEUES"] = "16"
    paths = [os.path.join(ROOT, "plonk.c_amd"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests")]
    r = subprocess.run([sys.executable, "-c", _CHILD, *paths], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return [l.split() for l in r.stdout.splitlines() if l[:1] in "23"]


@pytest.mark.parametrize("variant,what", [(1, "helper: chains_dev without done= ordering"),
                                          (2, "rank 0: rounds_ext_dev without the ready= wait")])
def test_missing_ordering_is_caught(variant, what):
    """the same stand-in run against a build with one hand-off ordering removed gives wrong proof
    bytes at both world sizes (and the real build, in the same child form, gives the right ones)"""
    lib = os.path.join(ROOT, "plonk.c_amd", "build", "diag", "libplonkhip_drop%d.so" % variant)
    assert os.path.exists(lib), "diagnostic build missing: make -C plonk.c_amd diag (__graft_entry__.build does)"
    rows = _child(lib)
    assert len(rows) == 2
    for world, got, want in rows:
        assert got != want, "%s not caught at world %s" % (what, world)
    for world, got, want in _child(os.path.join(ROOT, "plonk.c_amd", "libplonkhip.so")):
        assert got == want, world
