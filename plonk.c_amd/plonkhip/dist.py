"""Multi-GPU MSM by point-range sharding (reference srs_eval_at_s,
src/srs.h:53-68).

One process per GPU.  Rank r owns points [lo_r, hi_r) of the SRS and the matching
coefficients; its MSM kernel leaves a partial discrete log (0..101) and an irregular-input
count in a result record.  Because E(F101) is cyclic of order 102 (the logs are an exact group
isomorphism on canonical encodings), the commitment is EXP[(sum over ranks of partial logs) mod
102]: the only exchange is ONE collective SUM of (log, irregular) int32 pairs -- a whole batch of
MSMs shares it -- followed by a local map log -> point.  Any shard order gives the same bits.

Irregular encodings (off-curve points, coordinates >= 101, bad flag bytes) are not group
elements: the reference still folds them with its raw formulas, serially and order-dependently,
so they cannot be split into shards.  When any rank reports one for an MSM, the shards of that
MSM are all-gathered (in rank order, i.e. point order) and every rank re-runs the exact serial
fold over the whole range -- the single-GPU fallback, now over the gathered bytes.

The collectives go through torch.distributed (RCCL over xGMI on the GPU box, gloo in the CPU
tests).  The compute is injected: the GPU path (`gpu_ops`) calls libplonkhip; the CPU tests
pass the oracle.  The same `sharded_msm` runs in bench.py and in tests/test_dist_cpu.py.
"""

GROUP_ORDER = 102


def shard_range(n, rank, world):
    """Contiguous, balanced point range [lo, hi) of rank (the first n % world ranks get one
    extra point)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world %r/%r" % (rank, world))
    base, extra = divmod(int(n), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def combine_partials(partials, group=None):
    """partials: int32/int64 tensor [batch, 2] of this rank's (partial log, irregular count).
    ONE all-reduce SUM over the group (in place).  Returns (logs mod 102, irregular flags) as
    tensors [batch] on the same device."""
    dist = _dist()
    if dist is not None and dist.get_world_size(group) > 1:
        dist.all_reduce(partials, op=dist.ReduceOp.SUM, group=group)
    return partials[:, 0] % GROUP_ORDER, partials[:, 1] != 0


def gather_shards(points, scalars, n, group=None):
    """All-gather the shards of one MSM in rank order: (points[3n], scalars[n]) uint8 tensors
    of the whole range on every rank.  points/scalars: this rank's shard (flat uint8)."""
    import torch
    dist = _dist()
    if dist is None or dist.get_world_size(group) == 1:
        return points, scalars
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    width = -(-n // world)                       # max shard length (sizes differ by <= 1)
    lo, hi = shard_range(n, rank, world)
    buf = torch.zeros(4 * width, dtype=torch.uint8, device=points.device)
    buf[:3 * (hi - lo)] = points[:3 * (hi - lo)]
    buf[3 * width:3 * width + hi - lo] = scalars[:hi - lo]
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    pts, sc = [], []
    for r in range(world):
        a, b = shard_range(n, r, world)
        pts.append(parts[r][:3 * (b - a)])
        sc.append(parts[r][3 * width:3 * width + b - a])
    return torch.cat(pts), torch.cat(sc)


def finish_sharded(partials, n, ops, shard_of, group=None):
    """Finish a batch of sharded MSMs from this rank's partials (int32 tensor [batch, 2]:
    partial log, irregular count): ONE all-reduce SUM, the log -> point map, and the gathered
    serial fold for every MSM some rank flagged.  shard_of(b) -> (shard points, shard scalars)
    of MSM b (only called for flagged MSMs).  Returns (G1 results, identical on every rank: a
    uint8 tensor [batch, 4] of {x, y, infinite, 0} on the partials' device; number of MSMs that
    took the gathered serial fold)."""
    import torch
    logs, irr = combine_partials(partials, group)
    out = ops.exp(logs)
    flagged = torch.nonzero(irr).flatten().tolist()       # same decision on every rank
    for b in flagged:
        sp, ss = shard_of(b)
        pts, sc = gather_shards(sp, ss, n, group)
        out[b, :3] = torch.tensor(list(ops.fold(pts, sc)), dtype=torch.uint8, device=out.device)
    return out, len(flagged)


def g1_bytes(out):
    """list of 3-byte G1 encodings from finish_sharded's tensor"""
    host = out.cpu().numpy()
    return [bytes(host[b, :3]) for b in range(host.shape[0])]


def sharded_msm(shard_points, shard_scalars, n, ops, group=None):
    """A batch of MSMs of n points each, point-range sharded over the group.

    shard_points[b] / shard_scalars[b]: this rank's shard of MSM b (flat uint8 tensors of
    3 (hi - lo) / (hi - lo) bytes, [lo, hi) = shard_range(n, rank, world)).
    ops: `partials(shard_points, shard_scalars) -> int32 tensor [batch, 2]` (log, irregular),
    `exp(logs) -> uint8 tensor [batch, 4]` ({x, y, infinite, 0}), `fold(points, scalars) -> 3
    bytes` (the exact serial fold, src/srs.h:59-66).  See finish_sharded for the result."""
    part = ops.partials(shard_points, shard_scalars)
    return finish_sharded(part, n, ops, lambda b: (shard_points[b], shard_scalars[b]), group)


class gpu_ops:
    """libplonkhip behind `sharded_msm`: one batched kernel launch over the shards (result
    records on the device), a batched log -> point map, the serial fold for irregular MSMs."""

    def __init__(self, hip, stream=None):
        self.hip = hip
        self.stream = stream

    def launch(self, points0, points_stride, scalars0, scalars_stride, m, batch, records):
        """ONE batched launch: MSM b over m points at points0 + b points_stride (bytes) and
        scalars0 + b scalars_stride; result record b = records[b] (re-armed by the kernel)."""
        self.hip.msm_g1_batch_dev(points0, points_stride, scalars0, scalars_stride, m, batch, records[0],
                                  self.stream)

    def records_to_partials(self, records):
        """int32 tensor [batch, 2] = (partial log, irregular count) of result records."""
        import torch
        words = records.view(torch.int32)
        hip = self.hip
        return torch.stack([words[:, hip.MSM_LOG_OFFSET // 4], words[:, hip.MSM_IRREGULAR_OFFSET // 4]],
                           1).contiguous()

    def partials(self, shard_points, shard_scalars):
        import torch
        batch = len(shard_points)
        m = shard_scalars[0].numel()
        res = torch.zeros((batch, self.hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=shard_scalars[0].device)
        ps = shard_points[1].data_ptr() - shard_points[0].data_ptr() if batch > 1 else 0
        ss = shard_scalars[1].data_ptr() - shard_scalars[0].data_ptr() if batch > 1 else 0
        strided = batch == 1 or (ps > 0 and ss > 0 and all(
            shard_points[b].data_ptr() == shard_points[0].data_ptr() + b * ps and
            shard_scalars[b].data_ptr() == shard_scalars[0].data_ptr() + b * ss for b in range(batch)))
        if strided:                              # one launch over the whole batch
            self.launch(shard_points[0], ps, shard_scalars[0], ss, m, batch, res)
        else:
            for b in range(batch):
                self.hip.msm_g1_dev(shard_points[b], shard_scalars[b], m, res[b], self.stream)
        return self.records_to_partials(res)

    def exp(self, logs):
        import torch
        logs = logs.to(torch.int32).contiguous()
        out4 = torch.zeros((logs.numel(), 4), dtype=torch.uint8, device=logs.device)
        self.hip.msm_finalize_dev(logs, logs.numel(), 1, out4, self.stream)
        return out4

    def fold(self, points, scalars):
        import torch
        res = torch.zeros(self.hip.MSM_RESULT_BYTES, dtype=torch.uint8, device=scalars.device)
        self.hip.msm_g1_serial_dev(points, scalars, scalars.numel(), res, self.stream)
        return bytes(res[self.hip.MSM_G1_OFFSET:self.hip.MSM_G1_OFFSET + 3].cpu().numpy())


# ---- one proof strong-scaled over up to 3 ranks (bench.py prove_split_component)
CHAIN_T2, CHAIN_T3 = 1, 2   # PLK_CHAIN_T2 / PLK_CHAIN_T3: t_2 = (A2 B2)(C2 z), t_3 = (A3 B3)(C3 z(omega x))


def chain_assignment(world):
    """helper rank -> the round-3 chains it computes (src/plonk.h:432-434, 471-473): at N = 2 rank 1
    takes t_3 (rank 0 keeps t_2 with its (a b) q_m sum group); at N >= 3 rank 1 t_2 and rank 2 t_3;
    other ranks idle."""
    if world < 2:
        return {}
    return {1: CHAIN_T3} if world == 2 else {1: CHAIN_T2, 2: CHAIN_T3}


def split_proof_step(prover, polys, chal, rnd, bufs, rank, world, stream=None, via_host=False, group=None,
                     comm=None):
    """One strong-scaled proof.  Helpers: prover.chains_dev(...) into bufs, then send the bytes to
    rank 0; rank 0: receive them into bufs, then prover.rounds_ext_dev(...) reads them after the
    receive.  `stream`: torch's current stream (the one a device receive's wait() orders and a
    device send follows; None = the null stream).  bufs = {CHAIN_T2: tensor, CHAIN_T3: tensor}
    (plk_prover_chain_bytes each, on this rank's device).  via_host: move the bytes through host
    memory (gloo, which has no device send / receive).  comm: the torch.distributed-like module to
    use (default: torch.distributed itself; tests inject a stand-in with RCCL's stream semantics).
    Returns the proof bytes on rank 0, None elsewhere; every rank's part is complete on return.

    Stream ordering of the device branch (RCCL): a receive's wait() makes `stream` wait for the
    bytes, and rounds_ext_dev(ready=stream) makes the prover's stream wait for `stream` before its
    numerator (the only reader of the chains); on a helper, chains_dev(done=stream) makes `stream`
    wait for the chains, so the send (ordered behind `stream`) reads finished products."""
    import torch
    dist = comm if comm is not None else _dist()
    assign = chain_assignment(world)
    if rank == 0:
        reqs, host = [], []
        for r, m in sorted(assign.items()):
            for c in (CHAIN_T2, CHAIN_T3):
                if m & c:
                    if via_host:
                        h = torch.empty(bufs[c].numel(), dtype=torch.uint8)
                        dist.recv(h, src=r, group=group)
                        host.append((c, h))
                    else:
                        reqs.append(dist.irecv(bufs[c], src=r, group=group))
        for q in reqs:
            q.wait()                         # (RCCL: the current stream waits for the receive)
        for c, h in host:
            bufs[c].copy_(h)
        got = 0
        for m in assign.values():
            got |= m
        return prover.rounds_ext_dev(polys, chal, rnd, got, bufs[CHAIN_T2], bufs[CHAIN_T3], ready=stream)
    m = assign.get(rank, 0)
    if m:
        prover.chains_dev(polys, chal, rnd, m, bufs[CHAIN_T2] if m & CHAIN_T2 else None,
                          bufs[CHAIN_T3] if m & CHAIN_T3 else None, done=stream)
        for c in (CHAIN_T2, CHAIN_T3):
            if m & c:
                dist.send(bufs[c].cpu() if via_host else bufs[c], dst=0, group=group)
        if bufs[CHAIN_T2].is_cuda:
            torch.cuda.synchronize()
    return None
