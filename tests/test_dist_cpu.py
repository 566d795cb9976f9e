"""Point-range sharded MSM over world_size 2 with gloo on CPU: shards + one SUM all-reduce of
partial logs must reproduce the single-device result bit for bit (the partials come from
the oracle here; on the GPU box they come from libplonkhip)."""
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


def _worker(rank, world, port, n, batch, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "plonk.c_amd"), os.path.join(root, "oracle"), os.path.join(here, "golden")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import gen as g
    from plonkhip.dist import sharded_msm_logs
    from pyoracle import Oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = Oracle()
    inputs = [g.msm_inputs(100 + b, n, "full") for b in range(batch)]

    def partial(lo, hi, b):
        pts, sc = inputs[b]
        return orc.msm_dlog(pts[lo:hi], sc[lo:hi])[0]

    logs = sharded_msm_logs(n, rank, world, partial, batch=batch)
    q.put((rank, [orc.dlog_exp(int(v)).hex() for v in logs]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_msm_matches_single_device(oracle, world):
    n, batch = 10007, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [oracle.msm(*gen.msm_inputs(100 + b, n, "full")).hex() for b in range(batch)]
    for r in range(world):
        assert got[r] == want


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
