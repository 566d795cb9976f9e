"""In-process multi-device MSM through the C ABI (plk_init_devices, plonk.c_amd/csrc/shards.hip;
SURVEY 8(b) plk_init(n_gpus), 8(e) point-range sharding), rehearsed on the one GPU of a test box
by naming device 0 several times: every shard has its own stream, staging, host thread, result
record and SRS cache, exactly as on N devices.  The reference caller is srs_eval_at_s
(src/srs.h:53-68): results must equal the reference's goldens and the oracle fold, including the
irregular encodings (which fall back to the whole-input serial fold on the primary device)."""
import os
import subprocess

import numpy as np
import pytest

import gen
from conftest import ROOT, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture
def shards(hip):
    def use(ids, shard_min=None):
        hip.init_devices(ids)
        if shard_min is not None:
            hip.set_option("MSM_SHARD_MIN", shard_min)
    yield use
    hip.set_option("MSM_SHARD_MIN", 1 << 16)
    hip.init_devices([0])
    assert hip.devices() == [0]


@pytest.mark.parametrize("ids", [[0, 0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_goldens_through_shards(hip, shards, ids):
    """every reference golden (small cases incl. irregular encodings with the shard minimum at 1,
    and the seeded large inputs up to 2^22 points) through N shards"""
    shards(ids, 1)
    assert hip.devices() == ids
    g = load_golden("msm.json")
    for c in g["cases"]:
        assert hip.msm_g1(bytes.fromhex(c["points"]), bytes.fromhex(c["scalars"])).hex() == c["out"], c
    hip.set_option("MSM_SHARD_MIN", 1 << 16)
    for c in g["large"]:
        pts, sc = gen.msm_inputs(c["seed"], c["n"], c["kind"])
        assert hip.msm_g1(pts, sc).hex() == c["out"], (c["n"], c["kind"])


def test_sizes_and_irregular_vs_oracle(hip, oracle, shards):
    """sizes below, at and around the shard count (empty shards), every input kind, and
    irregular encodings placed in the middle of one shard or at a shard boundary"""
    shards([0, 0, 0], 1)
    for n in (1, 2, 3, 4, 5, 7, 100, 1000, 4099, 70001):
        for kind in ("subgroup", "full", "bytes"):
            pts, sc = gen.msm_inputs(300 + n, n, kind)
            assert hip.msm_g1(pts, sc) == oracle.msm(pts, sc), (n, kind)
    n = 30000
    pts, sc = gen.msm_inputs(17, n, "subgroup")
    for at in (5, n // 3, n // 3 - 1, n - 1):
        bad = np.frombuffer(pts, np.uint8).copy().reshape(-1, 3)
        bad[at] = (7, 7, 0)                              # off the curve
        assert hip.msm_g1(bad.tobytes(), sc) == oracle.msm(bad.tobytes(), sc), at


def test_srs_cache_follows_the_prover_pattern(hip, oracle, shards):
    """one SRS array, commitments of lengths n+2 / n+3 alternating (shard boundaries move by a
    point: the cached ranges are extended, not re-uploaded), then bytes changed in place at the
    same pointer (the memcmp catches them)"""
    shards([0, 0, 0, 0])
    n = 1 << 18
    srs, _ = gen.msm_inputs(5, n + 8, "subgroup")
    srs = np.frombuffer(srs, np.uint8).copy()
    rng = np.random.default_rng(1)
    for ln in (n + 2, n + 3, n + 2, n + 3, n + 5, n):
        sc = rng.integers(0, 17, ln, dtype=np.uint8)
        assert hip.msm_g1(srs[:3 * ln], sc) == oracle.msm(srs[:3 * ln].tobytes(), sc.tobytes()), ln
    sc = rng.integers(0, 17, n + 2, dtype=np.uint8)
    view = srs[:3 * (n + 2)]
    assert hip.msm_g1(view, sc) == oracle.msm(view.tobytes(), sc.tobytes())
    pts = srs.reshape(-1, 3)
    for at in (n // 2, n // 4 + 1, 3):                  # other canonical points, same array and pointer
        pts[at] = pts[(at * 7 + 1) % n]
        assert hip.msm_g1(view, sc) == oracle.msm(view.tobytes(), sc.tobytes()), at


def test_back_to_one_device_and_bad_lists(hip, shards):
    shards([0, 0])
    assert hip.devices() == [0, 0]
    hip.init_devices([0])
    assert hip.devices() == [0]
    for bad in ([], [0] * 17, [0, 999]):
        with pytest.raises(hip.PlonkHipError):
            hip.init_devices(bad)
    assert hip.devices() == [0]


SHARDED = os.path.join(ROOT, "oracle", "_ref", "dropin_tests_sharded")


@pytest.mark.parametrize("name", ["plonk", "srs"])
def test_reference_tests_through_shards(name):
    """The reference's own unmodified plonk-test.c / srs-test.c built against the drop-in with the
    shard minimum at 1 point (oracle/Makefile dropin-tests-sharded: -DPLK_DROPIN_SHARD_MIN=1),
    run with PLK_DEVICE=0,0,0: every srs_eval_at_s of every proof goes through three shards."""
    path = os.path.join(SHARDED, name + "-test")
    assert os.path.exists(path), "%s missing: `make -C oracle ref` where /root/reference exists" % path
    r = subprocess.run([path], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PLK_DEVICE="0,0,0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
