"""Source guard for a gfx950 compiler miscompile (ROCm 7.2 clang 22, pinned by tools/swar_probe.hip).

The AMDGPU dot4 combine rewrites an add chain of products c_t * (w_t & 0x00FF00FF) -- two byte
lanes per 32-bit word (SWAR) -- into v_dot4_u32_u8 over byte 0 only, silently dropping the upper
lane's terms (probe: 1,973,430 of 4,194,304 bytes wrong; the same arithmetic with the masked word
made opaque by an empty asm is exact).  Products of genuine single bytes (x & 0xFF), which every
kept kernel uses, are what the instruction computes and stay exact.  This test keeps multi-byte
lane masks out of multiplicative expressions in the device sources."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "plonk.c_amd", "csrc")

# a hex constant with 0xFF bytes separated by zero bytes (0x00FF00FF, 0xFF00FF): byte lanes.  Contiguous
# masks (0xFF, 0xFFFF, 0xFFFF0000) select one field and do not match.
LANE_MASK = re.compile(r"0x0*ff(?:00)+ff(?:00|ff)*u?\b", re.IGNORECASE)
# a product: `*` or the 24-bit multiply intrinsics (round 4's first lc16_swar had the mask inside
# __umul24 and passed a `*`-only check; it now goes through prove.hip's lanes02 / lanes13, whose
# empty asm keeps the combine from seeing the mask)
MUL = re.compile(r"\*|__u?mul24|__builtin_amdgcn_mul_u?24")


def test_no_swar_lane_masks_in_products():
    hits = []
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith((".hip", ".h")):
            continue
        with open(os.path.join(CSRC, name)) as f:
            for no, line in enumerate(f, 1):
                code = line.split("//")[0]
                if LANE_MASK.search(code) and MUL.search(code):
                    hits.append("%s:%d: %s" % (name, no, line.strip()))
    assert not hits, "SWAR lane mask in a product (see tools/swar_probe.hip):\n" + "\n".join(hits)


def test_lane_mask_pattern():
    assert LANE_MASK.search("lo += c * (w & 0x00FF00FFu);")
    assert LANE_MASK.search("x * (y & 0xff00ff)")
    assert not LANE_MASK.search("(d & 0xFFu) * c")
    assert not LANE_MASK.search("v & 0xFFFFu")
    assert MUL.search("E += __umul24(cf, w & 0x00FF00FFu);")


def test_guard_defeats_the_combine():
    """The empty-asm guard still keeps this compiler from forming the byte-0-only v_dot4
    (compile-only: tools/swar_dot4_check.sh on tools/swar_dot4_repro.hip)."""
    import shutil
    import subprocess
    import pytest
    if not os.path.exists("/opt/rocm/bin/hipcc") or not shutil.which("awk"):
        pytest.skip("no hipcc")
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "swar_dot4_check.sh")], capture_output=True,
                         text=True, timeout=300, check=True).stdout.split("\n")
    res = dict(l.split(" ", 1) for l in out if l.strip())
    assert res["swar_guarded"] == "dot4=0 mask=4", out


def _local_includes(path):
    """the csrc-relative names a source file pulls in with #include "..." (transitively)"""
    seen, todo = set(), [path]
    while todo:
        with open(os.path.join(CSRC, todo.pop())) as f:
            for line in f:
                m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
                if m:
                    name = os.path.normpath(m.group(1))
                    if name not in seen:
                        seen.add(name)
                        if os.path.exists(os.path.join(CSRC, name)) and not name.startswith(".."):
                            todo.append(name)
    return seen


def test_makefile_hdr_lists_every_local_include():
    """an edit to any header a kernel includes must rebuild its object (round 4 missed
    plk_msm_finish.h: msm.o / prove.o went stale on a finish-code edit)"""
    with open(os.path.join(ROOT, "plonk.c_amd", "Makefile")) as f:
        mk = f.read()
    hdr = re.search(r"^HDR\s*:=\s*(.*)$", mk, re.M).group(1).split()
    hdr = {os.path.normpath(h[len("csrc/"):]) if h.startswith("csrc/") else os.path.normpath(os.path.join("..", h))
           for h in hdr}
    missing = []
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".h")):
            for inc in _local_includes(name):
                if inc not in hdr:
                    missing.append("%s includes %s" % (name, inc))
    assert not missing, "plonk.c_amd/Makefile HDR misses:\n" + "\n".join(missing)


def test_pmc_hash_covers_msm_headers():
    """bench.py's kernel_source_hash (which invalidates the committed PMC traffic record) must
    cover every csrc header msm.hip includes"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    want = {"msm.hip"} | {i for i in _local_includes("msm.hip") if not i.startswith("..")}
    assert want <= set(bench.MSM_SOURCES), sorted(want - set(bench.MSM_SOURCES))
