"""Point-range sharded MSM over gloo on CPU (world 2 and 3): `plonkhip.dist.sharded_msm` -- the
exact function bench.py runs over RCCL -- must reproduce the single-device serial fold bit for
bit (reference srs_eval_at_s, src/srs.h:53-68), including MSMs whose irregular encodings force
the gathered serial fold.  The per-shard partials come from the oracle here; on the GPU box they
come from libplonkhip (`plonkhip.dist.gpu_ops`)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import gen


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(n, batch, irregular_at):
    out = []
    for b in range(batch):
        pts, sc = gen.msm_inputs(100 + b, n, "full")
        pts = pts.copy()
        if b in irregular_at:                     # an off-curve point inside the given index
            pts[irregular_at[b]] = (5, 5, 0)
        out.append((pts, sc))
    return out


class OracleOps:
    """sharded_msm's compute, from the CPU oracle (test infrastructure)."""

    def __init__(self, orc):
        self.orc = orc

    def partials(self, shard_points, shard_scalars):
        import torch
        rows = []
        for p, s in zip(shard_points, shard_scalars):
            log, _ = self.orc.msm_dlog(p.numpy(), s.numpy())
            rows.append([0, 1] if log is None else [log, 0])
        return torch.tensor(rows, dtype=torch.int32)

    def exp(self, logs):
        import torch
        return torch.tensor([list(self.orc.dlog_exp(int(v))) + [0] for v in logs], dtype=torch.uint8)

    def fold(self, points, scalars):
        return self.orc.msm(points.numpy(), scalars.numpy())


def _worker(rank, world, port, n, batch, irregular_at, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "plonk.c_amd"), os.path.join(root, "oracle"), here, os.path.join(here, "golden")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from plonkhip.dist import g1_bytes, shard_range, sharded_msm
    from pyoracle import Oracle
    from test_dist_cpu import OracleOps, _inputs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    sp, ss = [], []
    for pts, sc in _inputs(n, batch, irregular_at):
        sp.append(torch.from_numpy(pts[lo:hi].reshape(-1).copy()))
        ss.append(torch.from_numpy(sc[lo:hi].copy()))
    out, folded = sharded_msm(sp, ss, n, OracleOps(Oracle()))
    q.put((rank, [o.hex() for o in g1_bytes(out)], folded))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, n, batch, irregular_at):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, batch, irregular_at, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, out, folded = q.get(timeout=120)
        got[r] = (out, folded)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_msm_matches_single_device(oracle, world):
    n, batch = 10007, 3
    got = _run(world, n, batch, {})
    want = [oracle.msm(p, s).hex() for p, s in _inputs(n, batch, {})]
    for r in range(world):
        assert got[r] == (want, 0)


@pytest.mark.parametrize("world,late", [(2, 1), (8, 5)])
def test_irregular_point_in_a_later_shard(oracle, world, late):
    """an off-curve point in rank `late`'s shard of MSM 1 (and in rank 0's of MSM 2): those MSMs take
    the gathered serial fold (the 8-way gather at the driver's largest world size) and still equal
    the reference fold; MSM 0 stays on the log path"""
    from plonkhip.dist import shard_range
    n, batch = 4099, 3
    lo1, _ = shard_range(n, late, world)
    irregular_at = {1: lo1 + 17, 2: 3}
    got = _run(world, n, batch, irregular_at)
    want = [oracle.msm(p, s).hex() for p, s in _inputs(n, batch, irregular_at)]
    for r in range(world):
        assert got[r] == (want, 2)


def test_shard_ranges_cover_exactly():
    from plonkhip.dist import shard_range
    for n in (0, 1, 7, 1 << 22, (1 << 22) + 5):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


# ---- the strong-scaled proof's choreography (plonkhip.dist.split_proof_step, what bench.py's
# prove_split_component runs over RCCL) with a stand-in prover: helpers fill their chain buffers
# with known bytes, rank 0's "proof" is a digest of the chains it received
_CHAIN_LEN = 4099


def _chain_bytes(c, chal):
    import torch
    return (torch.arange(_CHAIN_LEN, dtype=torch.int64) * (7 * c + chal[0]) % 251).to(torch.uint8)


class MockProver:
    def chains_dev(self, polys, chal, rnd, which, t2=None, t3=None, done=None):
        for c, buf in ((1, t2), (2, t3)):
            if which & c:
                buf.copy_(_chain_bytes(c, chal))

    def rounds_ext_dev(self, polys, chal, rnd, which, t2=None, t3=None, ready=None):
        import hashlib
        h = hashlib.sha256(bytes([which]))
        for c, buf in ((1, t2), (2, t3)):
            if which & c:
                h.update(buf.numpy().tobytes())
        return h.digest()


def _split_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "plonk.c_amd"))
    sys.path.insert(0, here)
    import torch
    import torch.distributed as dist

    from plonkhip.dist import split_proof_step
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from test_dist_cpu import MockProver
    bufs = {c: torch.zeros(_CHAIN_LEN, dtype=torch.uint8) for c in (1, 2)}
    outs = [split_proof_step(MockProver(), [], [5, 1, 2, 3, 4], [0] * 9, bufs, rank, world, via_host=True)
            for _ in range(2)]
    q.put((rank, [o.hex() if o is not None else None for o in outs]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_split_proof_choreography(world):
    """rank 1 (N = 2: t_3; N >= 3: t_2) and rank 2 (t_3) send their chains, rank 0 proves with
    exactly those, the other ranks idle; two proofs back to back keep the sends and receives
    paired"""
    import hashlib

    from plonkhip.dist import chain_assignment
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    union = 0
    for m in chain_assignment(world).values():
        union |= m
    assert union == (2 if world == 2 else 3)
    h = hashlib.sha256(bytes([union]))
    for c in (1, 2):
        if union & c:
            h.update(_chain_bytes(c, [5]).numpy().tobytes())
    assert got[0] == [h.digest().hex()] * 2
    assert all(got[r] == [None, None] for r in range(1, world))
