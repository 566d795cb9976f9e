"""The C-ABI boundary without a GPU: libplonkhip.so loads, exports exactly what
include/plonkhip.h declares, fails loudly (no CPU fallback) when no device is present, and
the drop-in headers compile -- standalone and under the reference's own plonk.h."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

INCLUDE = os.path.join(ROOT, "include")
PKG = os.path.join(ROOT, "plonk.c_amd")
REF_SRC = "/root/reference/src"


def declared_symbols():
    txt = open(os.path.join(INCLUDE, "plonkhip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(plk_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    import plonkhip
    lib = plonkhip.lib()
    decl = declared_symbols()
    assert len(decl) >= 15
    for s in decl:
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", plonkhip.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (plk_\w+)", out))
    assert exported == set(decl)
    assert set(plonkhip.SIGNATURES) == set(decl)


def test_library_is_gfx950_code():
    """The fat binary embedded in libplonkhip.so carries gfx950 code objects (and nothing
    else: no other targets, no host fallback)."""
    import plonkhip
    data = open(plonkhip.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_no_cpu_fallback_without_gpu():
    import plonkhip
    if plonkhip.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(plonkhip.PlonkHipError) as e:
        plonkhip.msm_g1([1, 2, 0], [1])
    assert e.value.code == plonkhip.PLK_ERR_NODEV
    with pytest.raises(plonkhip.PlonkHipError):
        plonkhip.poly_mul([1, 2], [3, 4])


def test_init_devices_without_gpu():
    """plk_init_devices: a malformed list is PLK_ERR_ARG before any device query; with no device
    a valid list is PLK_ERR_NODEV (no CPU fallback); plk_devices reports nothing initialised."""
    import plonkhip as h
    for bad in ([], [0] * 17):
        with pytest.raises(h.PlonkHipError) as e:
            h.init_devices(bad)
        assert e.value.code == h.PLK_ERR_ARG
    if h.device_count() == 0:
        with pytest.raises(h.PlonkHipError) as e:
            h.init_devices([0, 0])
        assert e.value.code == h.PLK_ERR_NODEV
        assert h.devices() == []


def test_host_argument_checks():
    import plonkhip
    with pytest.raises(ValueError):
        plonkhip.msm_g1([1, 2, 0, 1], [1])
    with pytest.raises(ValueError):
        plonkhip.srs_eval_at_s([1, 2, 0], [1, 1])


def test_options_without_gpu():
    """plk_set_option / plk_get_option (the library's only switches besides PLK_DEVICE) work with
    no device; defaults are the production settings; out-of-range values and unknown options
    are refused; the library source reads no other environment variable."""
    import plonkhip as h
    defaults = {"TINY_CALLS": 1, "PROVE_SYNC": 0, "POLY_BLOCK_L": 0, "POLY_BLOCK_S": 0, "NTT_F29": 1,
                "NTT_SHARE": 1, "NTT_SHARED_FIX": 1, "NTT_T13_MIN_K": 21, "NTT_CENTER_BLOCKS": 0,
                "MSM_HALF": 1, "MSM_SHARD_MIN": 1 << 16, "NTT_CENTER_SUM": 1, "MSM_HOST_LANES": 4,
                "PROVE_DERIVE_T2A": 2, "NTT_TABLE_SHARE": 1, "NTT_LAUNCH_LOG": 0,
                "PROVE_FUSE_DIV": 0, "PROVE_SRS_LOGS": 1, "PROVE_PACK_FUSE": 1, "PROVE_EARLY_COMMITS": 1,
                "PROVE_EVAL_AGG": 1, "PROVE_GRAPH": 0}
    for k, v in defaults.items():
        assert h.get_option(k) == v, k
    with h.options(NTT_SHARED_FIX=2, POLY_BLOCK_L=4096, POLY_BLOCK_S=513):
        assert h.get_option("NTT_SHARED_FIX") == 2 and h.get_option("POLY_BLOCK_S") == 513
    assert h.get_option("NTT_SHARED_FIX") == 1 and h.get_option("POLY_BLOCK_L") == 0
    for k, v in (("NTT_SHARED_FIX", 3), ("NTT_T13_MIN_K", 12), ("POLY_BLOCK_S", 3670017), (99, 0), (0, 0)):
        with pytest.raises(h.PlonkHipError) as e:
            h.set_option(k, v)
        assert e.value.code == h.PLK_ERR_ARG
    assert h.get_option(99) == -1
    csrc = os.path.join(PKG, "csrc")
    envs = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")):
            envs |= set(re.findall(r'getenv\("(\w+)"\)', open(os.path.join(csrc, f)).read()))
    assert envs == {"PLK_DEVICE"}


def test_split_prover_exports_without_gpu():
    """plk_prover_attach_helpers / plk_prover_helpers / plk_prover_rounds_multi_dev (one proof over
    the plk_init_devices list from C) refuse a NULL prover and bad counts before touching a device"""
    import ctypes as C

    import plonkhip as h
    lib = h.lib()
    assert lib.plk_prover_attach_helpers(None, 1) == h.PLK_ERR_ARG
    assert lib.plk_prover_attach_helpers(None, 3) == h.PLK_ERR_ARG
    assert lib.plk_prover_helpers(None) == 0
    chal, rnd, out = (C.c_uint8 * 5)(), (C.c_uint8 * 9)(), (C.c_uint8 * 34)()
    polys = (C.c_void_p * 13)()
    assert lib.plk_prover_rounds_multi_dev(None, polys, 1, chal, rnd, 0, out) == h.PLK_ERR_ARG


def test_prover_measurement_exports_without_gpu():
    """plk_prover_profile_dev / plk_prover_launches / plk_prover_alg_bytes (the bench line's C5
    roofline) refuse a NULL prover or NULL outputs before touching a device"""
    import ctypes as C

    import plonkhip as h
    lib = h.lib()
    chal, rnd, out = (C.c_uint8 * 5)(), (C.c_uint8 * 9)(), (C.c_uint8 * 34)()
    polys = (C.c_void_p * 13)()
    ms = (C.c_double * 4)()
    k, o = C.c_int(), C.c_int()
    assert lib.plk_prover_profile_dev(None, polys, chal, rnd, 0, out, ms) == h.PLK_ERR_ARG
    assert lib.plk_prover_launches(None, polys, chal, rnd, 0, C.byref(k), C.byref(o)) == h.PLK_ERR_ARG
    assert lib.plk_prover_alg_bytes(None) == 0
    assert "plk_prover_profile_dev" in h.last_error() or "plk_prover_launches" in h.last_error()


def _gcc(args, **kw):
    return subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-I", INCLUDE] + args,
                          capture_output=True, text=True, **kw)


def test_dropin_headers_compile_and_link(tmp_path):
    src = tmp_path / "use.c"
    src.write_text('#include "prelude.h"\n'
                   "int main(void) {\n"
                   "  SRS srs = srs_create(f101(5), 5);\n"
                   "  HF c[] = {{1}, {2}, {3}};\n"
                   "  POLY p = poly_new(c, 3);\n"
                   "  G1 e = srs_eval_at_s(&srs, &p);\n"
                   "  POLY q = poly_mul(&p, &p);\n"
                   "  poly_free(&q); poly_free(&p); srs_free(&srs);\n"
                   "  return e.infinite ? 0 : 1;\n}\n")
    r = _gcc([str(src), "-L", PKG, "-lplonkhip", "-o", str(tmp_path / "use")])
    assert r.returncode == 0, r.stderr
    # two translation units including the headers link together (static inline, unlike
    # the reference's single-TU headers)
    (tmp_path / "a.c").write_text('#include "srs.h"\nG1 fa(void){ return g1_generator(); }\n')
    (tmp_path / "b.c").write_text('#include "srs.h"\nG1 fa(void);\nint main(void){ G1 g = fa(); '
                                  'return g.x.value == 1 ? 0 : 1; }\n')
    r = _gcc([str(tmp_path / "a.c"), str(tmp_path / "b.c"), "-L", PKG, "-lplonkhip",
              "-o", str(tmp_path / "ab")])
    assert r.returncode == 0, r.stderr


def test_struct_layouts(tmp_path):
    import plonkhip
    (tmp_path / "l.c").write_text('#include "prelude.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                                  "int main(void){ printf(\"%zu %zu %zu %zu %zu %zu %zu\", sizeof(G1), "
                                  "sizeof(HF), sizeof(GF), sizeof(plk_msm_result_t), "
                                  "offsetof(plk_msm_result_t, log), offsetof(plk_msm_result_t, irregular), "
                                  "offsetof(plk_msm_result_t, g1)); return 0; }\n")
    r = _gcc([str(tmp_path / "l.c"), "-o", str(tmp_path / "l")])
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(tmp_path / "l")], capture_output=True, text=True).stdout
    assert out == "3 1 1 %d %d %d %d" % (plonkhip.MSM_RESULT_BYTES, plonkhip.MSM_LOG_OFFSET,
                                         plonkhip.MSM_IRREGULAR_OFFSET, plonkhip.MSM_G1_OFFSET)


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources not present")
def test_reference_plonk_test_compiles_against_dropin(tmp_path):
    """The reference's unmodified plonk-test.c + plonk.h build with our headers pre-included
    (the drop-in mechanism); running it needs the GPU (tests/test_dropin_gpu.py)."""
    r = subprocess.run(["gcc", "-std=gnu11", "-w", "-include", os.path.join(INCLUDE, "prelude.h"),
                        "-I", INCLUDE, os.path.join(REF_SRC, "plonk-test.c"), "-L", PKG,
                        "-lplonkhip", "-o", str(tmp_path / "plonk-test")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", str(tmp_path / "plonk-test")], capture_output=True, text=True).stdout
    for sym in ("plk_poly_mul", "plk_msm_g1", "plk_poly_divide", "plk_poly_eval", "plk_matrix_inv", "plk_matrix_mul"):
        assert "U " + sym in nm, sym
