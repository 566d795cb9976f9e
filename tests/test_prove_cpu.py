"""CPU side of the prover row: the restatement oracle/prove_ref.py reproduces every reference
proof and rejection recorded in tests/golden/prove.json (so it can serve as the parity oracle
for the device prover at sizes the reference cannot run), and the ctypes mirrors of the
prover structs match the C header layout."""
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden
from prove_ref import Prover, ProveError, poly_eval


def _run(o, g, case):
    key = "short" if case["srs_n"] == 4 else str(case["srs_mode"])
    s = {k: bytes.fromhex(v) for k, v in g["setups"][key].items()}
    pr = Prover(o, s["g1s"], 4, s["h"], s["k1_h"], s["k2_h"], s["h_pows_inv"], s["z_h"])
    gt, cp, w = case["gates"], case["copies"], case["wires"]
    copies = [[(cp[8 * k + 2 * i], cp[8 * k + 2 * i + 1]) for i in range(4)] for k in range(3)]
    return pr.prove(gt[0:4], gt[4:8], gt[8:12], gt[12:16], gt[16:20], copies, w[0:4], w[4:8], w[8:12],
                    case["chal"], case["rand"])


def test_restated_prover_matches_reference_proofs(oracle):
    g = load_golden("prove.json")
    assert len(g["proofs"]) >= 20
    for case in g["proofs"]:
        assert _run(oracle, g, case).hex() == case["proof"], (case["chal"], case["srs_mode"])


def test_restated_prover_rejects_like_reference(oracle):
    g = load_golden("prove.json")
    for case in g["failures"]:
        if case["proof"] is None:
            with pytest.raises(ProveError):
                _run(oracle, g, case)
        else:
            assert _run(oracle, g, case).hex() == case["proof"]


def test_setup_matches_plonk_new():
    """h = omega^i, k1/k2 cosets, inverse Vandermonde and Z_H = x^4 - 1 from the fixture are
    the group facts they should be (plonk_new, src/plonk.h:53-118)."""
    s = {k: bytes.fromhex(v) for k, v in load_golden("prove.json")["setups"]["0"].items()}
    h = list(s["h"])
    assert h == [pow(4, i, 17) for i in range(4)]
    assert list(s["k1_h"]) == [2 * x % 17 for x in h] and list(s["k2_h"]) == [3 * x % 17 for x in h]
    V = np.array([[pow(h[r], c, 17) for c in range(4)] for r in range(4)])
    Hi = np.frombuffer(s["h_pows_inv"], np.uint8).reshape(4, 4).astype(np.int64)
    assert ((Hi @ V) % 17 == np.eye(4, dtype=np.int64)).all()
    assert list(s["z_h"]) == [16, 0, 0, 0, 1]
    for x in h:
        assert poly_eval(np.frombuffer(s["z_h"], np.uint8), x) == 0


def test_prover_struct_layout(tmp_path):
    import ctypes as C
    import plonkhip
    src = ('#include "plonkhip.h"\n#include <stdio.h>\n#include <stddef.h>\n'
           "int main(void){ printf(\"%zu %zu %zu %zu %zu\", sizeof(plk_plonk_desc_t), "
           "offsetof(plk_plonk_desc_t, z_h_len), offsetof(plk_plonk_desc_t, srs_len), "
           "sizeof(plk_circuit_t), offsetof(plk_circuit_t, c)); return 0; }\n")
    (tmp_path / "s.c").write_text(src)
    r = subprocess.run(["gcc", "-std=gnu11", "-I", ROOT + "/include", str(tmp_path / "s.c"), "-o",
                        str(tmp_path / "s")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(tmp_path / "s")], capture_output=True, text=True).stdout.split()
    D, Cc = plonkhip.PlonkDesc, plonkhip.Circuit
    assert [int(x) for x in out] == [C.sizeof(D), D.z_h_len.offset, D.srs_len.offset, C.sizeof(Cc), Cc.c.offset]
