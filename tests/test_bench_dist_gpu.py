"""The multi-rank bench path (what the driver's N = 2/4/8 runs execute, one process per GPU over
RCCL) rehearsed on the one GPU of a test box: two ranks over gloo sharing cuda:0, strong scaling
(each 2^22-point MSM split by point range, plonkhip.dist.finish_sharded).  The line must carry the
strong-scaling config and both correctness checks -- the first MSM against a single-GPU recompute
and the reference's own 2^22-point golden through the sharded path -- plus C5's replica leg (one
2^20-gate proof per rank, released together by a barrier, every rank's bytes checked), C5
strong-scaled (round 3's t_2 / t_3 chains on ranks 1 / 2, their bytes sent to rank 0) and the
MSM components named by the points a rank actually reads (2^21 per shard here)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_strong_scaling_line():
    """plain `python bench.py --gpus 2`, no external launcher: the bench starts its two ranks itself
    (torch.distributed.run as a child) and the line says n_gpus 2"""
    env = dict(os.environ, PLK_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--msm-batch", "8", "--rotate-mib", "160", "--components", "prove,msm", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints exactly one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["steps"] == 3
    assert d["config"]["points_per_gpu"] * 2 == d["config"]["points_per_msm"] == 1 << 22
    assert d["checks"] == {"first_msm_single_gpu_recompute": True, "golden_2^22_reference": True}
    assert d["irregular_inputs"] == 0 and d["value"] > 0
    c = d["components"]
    rep = c["prove_2^20_gates_replicas"]
    assert rep["gpus"] == 2 and rep["matches_oracle_all_ranks"] is True and rep["deterministic_all_ranks"] is True
    assert rep["ms_slowest_rank"] > 0
    sp = c["prove_2^20_gates_split"]
    assert sp["gpus"] == 2 and sp["matches_oracle"] is True and sp["same_as_single_gpu"] is True and sp["ms"] > 0
    # a shard is 2^21 points: no key may claim 2^22 for it
    assert "msm_2^21_one_per_launch" in c and "msm_2^21_8_per_launch" in c
    assert not any(k.startswith("msm_2^22") for k in c)
    assert "prove_2^20_gates" not in c            # the single-GPU C5 line is not repeated at N > 1


def _plain_bench_line(n, components, batch, rotate, steps=2, timeout=540):
    """`python bench.py --gpus n` exactly as the driver's scaling run starts it (no launcher: the bench
    spawns its n ranks), gloo so that n ranks share the one GPU of a test box; rank 0's line"""
    env = dict(os.environ, PLK_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps), "--warmup", "1",
           "--msm-batch", str(batch), "--rotate-mib", str(rotate), "--components", components, "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [4, 8])
def test_driver_scaling_world_sizes(n):
    """the world sizes the driver's N = 1, 2, 4, 8 scaling run uses, rehearsed on one
    GPU before the first 8-GPU node sees them: an n-way shard_range of every 2^22-point MSM (the 2^22
    reference golden through the n shards), n concurrent proof replicas each matching the recorded answer,
    and the strong-scaled proof over 3 ranks with ranks 3 .. n-1 idle through every one of its barriers."""
    d = _plain_bench_line(n, "prove,msm", batch=4, rotate=8)
    assert d["n_gpus"] == n and d["scaling"] == "strong" and d["config"]["parallelism"] == "dp%d" % n
    assert d["config"]["points_per_gpu"] * n == d["config"]["points_per_msm"] == 1 << 22
    assert d["checks"] == {"first_msm_single_gpu_recompute": True, "golden_2^22_reference": True}
    assert d["irregular_inputs"] == 0 and d["serial_fold_fallbacks"] == 0 and d["value"] > 0
    c = d["components"]
    rep = c["prove_2^20_gates_replicas"]
    assert rep["gpus"] == n and rep["matches_oracle_all_ranks"] is True and rep["deterministic_all_ranks"] is True
    sp = c["prove_2^20_gates_split"]
    assert sp["gpus"] == 3 and sp["matches_oracle"] is True and sp["same_as_single_gpu"] is True
    lab = "2^%d" % (22 - (n.bit_length() - 1))
    assert "msm_%s_one_per_launch" % lab in c and "msm_%s_8_per_launch" % lab in c


def test_three_rank_split_proof():
    """C5 strong-scaled over three ranks: rank 1 computes the t_2 chain, rank 2 the t_3 chain, rank
    0 the rest; the proof equals the single-GPU proof and the recorded answer.  Launched the way the
    driver launches N > 1 (torch.distributed.run around bench.py, WORLD_SIZE = --gpus)."""
    env = dict(os.environ, PLK_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", "29563", os.path.join(ROOT, "bench.py"),
           "--gpus", "3", "--steps", "2", "--warmup", "1", "--msm-batch", "4", "--rotate-mib", "96",
           "--components", "prove", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    sp = d["components"]["prove_2^20_gates_split"]
    assert sp["gpus"] == 3 and sp["matches_oracle"] is True and sp["same_as_single_gpu"] is True
    assert d["components"]["prove_2^20_gates_replicas"]["matches_oracle_all_ranks"] is True
