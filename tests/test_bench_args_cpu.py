"""bench.py's rank handling before any GPU work: `--gpus N` without a launcher
starts N ranks itself (torch.distributed.run as a child process), and a launcher's WORLD_SIZE that
disagrees with --gpus stops the run before torch -- let alone HIP -- is imported."""
import importlib.util
import os
import subprocess
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _poisoned_torch(tmp_path):
    """a PYTHONPATH entry whose `torch` raises on import: a run that gets past the rank check fails
    with this message instead of the check's"""
    d = tmp_path / "poison"
    (d / "torch").mkdir(parents=True)
    (d / "torch" / "__init__.py").write_text("raise ImportError('POISON: torch imported before the rank check')\n")
    return str(d)


def _run(tmp_path, args, world):
    env = dict(os.environ, PYTHONPATH=_poisoned_torch(tmp_path))
    env.pop("WORLD_SIZE", None)
    if world is not None:
        env["WORLD_SIZE"] = str(world)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=60)


def test_world_size_mismatch_exits_before_torch(tmp_path):
    r = _run(tmp_path, ["--gpus", "4", "--steps", "1"], world=2)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr, r.stderr
    assert "POISON" not in r.stderr                 # stopped before `import torch`


def test_world_size_match_proceeds_to_torch(tmp_path):
    # the control: a consistent launch gets past the check and reaches the (poisoned) torch import
    r = _run(tmp_path, ["--gpus", "2", "--steps", "1"], world=2)
    assert r.returncode != 0 and "POISON" in r.stderr, r.stderr


def test_bad_gpu_count_rejected(tmp_path):
    r = _run(tmp_path, ["--gpus", "0"], world=None)
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr and "POISON" not in r.stderr


def test_world_from_args():
    b = _bench()
    ns = lambda g: types.SimpleNamespace(gpus=g)  # noqa: E731
    assert b.world_from_args(ns(None), {}) == (1, False)
    assert b.world_from_args(ns(1), {}) == (1, False)
    assert b.world_from_args(ns(8), {}) == (8, True)          # no launcher: start the ranks
    assert b.world_from_args(ns(8), {"WORLD_SIZE": "8"}) == (8, False)
    assert b.world_from_args(ns(None), {"WORLD_SIZE": "4"}) == (4, False)
    try:
        b.world_from_args(ns(8), {"WORLD_SIZE": "1"})
        raise AssertionError("mismatch accepted")
    except SystemExit as e:
        assert "WORLD_SIZE=1" in str(e)


def test_rank_launch_cmd_is_the_driver_form():
    """the child is the command the driver itself uses for N > 1: one node, N processes, rendezvous
    on 127.0.0.1, this bench.py with the caller's own arguments"""
    b = _bench()
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = b.rank_launch_cmd(argv, 8, 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8" and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29999"
    j = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[j + 1:] == argv


def test_bench_source_has_no_exec():
    """the ranks are a child process: an exec from a process that may have touched the GPU is
    forbidden on this pool, and bench.py needs none"""
    with open(os.path.join(ROOT, "bench.py")) as f:
        src = f.read()
    assert "os.exec" not in src and "execv" not in src


def test_roofline_accounting_of_a_launch_plan():
    """plonkhip.roofline (shared by bench.py's C5 line and tools/ntt_roofline.py): the butterflies and
    bytes of each kind of NTT launch record, priced against the peak of its kind and field"""
    sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
    from plonkhip import roofline as RL
    pk = {"f29_dif_Gbfly_s": 6000.0, "f29_dit_Gbfly_s": 5000.0, "bb_dif_Gbfly_s": 4000.0, "bb_dit_Gbfly_s": 3000.0}
    fwd = {"kind": 0, "tb": 13, "m": 8, "k": 21, "n": 15, "per_block": 8, "units": 0, "field": 0}
    inv = {"kind": 1, "tb": 13, "m": 8, "k": 21, "n": 7, "per_block": 4, "units": 0, "field": 0}
    cen = {"kind": 2, "tb": 13, "m": 13, "k": 21, "n": 9, "per_block": 1, "units": 22, "field": 0}
    fix = {"kind": 3, "tb": 13, "m": 13, "k": 21, "n": 3, "per_block": 1, "units": 3, "field": 1}
    tiles, half = 1 << 8, 1 << 12
    assert RL.launch_butterflies(fwd) == tiles * 15 * 8 * half
    assert RL.launch_butterflies(inv) == tiles * 7 * 8 * half
    assert RL.launch_butterflies(cen) == tiles * 22 * 13 * half
    assert RL.launch_butterflies(fix) == tiles * 3 * 13 * half
    assert RL.launch_bytes(fwd) == (1 << 21) * 15 * 8 and RL.launch_bytes(cen) == (1 << 21) * 9 * 12
    assert RL.peak_bfly_s(0, 0, pk) == 6000e9 and RL.peak_bfly_s(1, 0, pk) == 5000e9
    assert RL.peak_bfly_s(3, 1, pk) == 4000e9
    assert abs(RL.peak_bfly_s(2, 0, pk) - 3 / (2 / 6000e9 + 1 / 5000e9)) < 1
    tot = RL.plan_roofline([fwd, inv, cen, fix], pk)
    want = sum(RL.launch_butterflies(r) / RL.peak_bfly_s(r["kind"], r["field"], pk) for r in (fwd, inv, cen, fix))
    assert tot["launches"] == 4 and abs(tot["roof_s"] - want) < 1e-15
    # the committed peak file parses
    assert RL.load_peaks(RL.PEAKS)["f29_dif_Gbfly_s"] > 1000
