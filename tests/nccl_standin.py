"""A torch.distributed stand-in with RCCL's stream semantics, for ONE process that plays every rank
on one GPU (tests/test_split_streams_gpu.py).  It exists so that the device branch of
plonkhip.dist.split_proof_step -- the branch an 8-GPU node takes over RCCL -- runs on a one-GPU box,
with the same ordering hazards:

* send(t): RCCL's send kernel runs on the communicator's own stream behind an event of the caller's
  CURRENT stream; it reads `t` when that stream gets there, not when send() returns.  Here: the side
  stream waits for an event of the current stream and copies `t` into a staging tensor (the "wire").
* irecv(t): the bytes land on the communicator's stream; work.wait() makes the CURRENT stream wait
  for them and returns at once (no host block).  Here: the side stream spins first (`delay` cycles
  of torch.cuda._sleep, so the bytes arrive late), then copies the staged bytes into `t`; wait()
  is current_stream().wait_event.

A consumer that does not order itself behind the current stream at the right point reads bytes
that are not there yet -- exactly what a missing ready= / done= ordering would do over RCCL.

What keeps a missing ordering from being hidden by timing or by stale memory:
* irecv poisons its target (0x05 bytes, finished before it returns), so an unordered read of it
  sees poison, not an earlier proof's bytes left in a reused allocation; the drop-1 diagnostic
  build likewise poisons its products and writes them ~20 ms later (prove.hip);
* before each helper's step the current stream spins (`delay` cycles): the helper's chains start
  behind it (plk_prover_chains_dev makes its stream wait for `done` first), and so does a send
  with no ordering -- which then copies while the chains run instead of after them;
* HIP multiplexes streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default), in order per
  queue: two streams that share one serialise in submission order and hide any race between
  them.  The negative test (tests/test_split_streams_gpu.py) runs in a child process with 16
  queues, more than the streams it creates, so every stream has its own;
* a stream's FIRST use waits for all work on the device (measured, tools/stream_probe.py: its
  hardware queue is created then), which would order a first send behind the chains: the side
  stream and every prover's stream are used once before the checked proof.
"""
import torch

DELAY_CYCLES = 20_000_000   # the receive's spin on the side stream (milliseconds of device time)


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class NcclSemantics:
    def __init__(self, delay=DELAY_CYCLES):
        self.side = torch.cuda.Stream()
        self.delay = delay
        self.wire = {}          # dst rank -> [(staged tensor, event after its copy)], in send order
        # a stream's first use waits for the whole device (HIP creates its hardware queue then:
        # tools/stream_probe.py), which would order the first send / receive behind everything
        with torch.cuda.stream(self.side):
            torch.zeros(1, device="cuda").add_(1)
        torch.cuda.synchronize()

    def send(self, t, dst, group=None):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.side.wait_event(ev)
        staged = torch.empty_like(t)
        with torch.cuda.stream(self.side):
            staged.copy_(t)
        staged.record_stream(self.side)
        done = torch.cuda.Event()
        done.record(self.side)
        self.wire.setdefault(dst, []).append((staged, done))

    def irecv(self, t, src, group=None):
        # (this stand-in serves rank 0's receives in send order; the choreography sends each chain once)
        staged, done = self.wire[0].pop(0)
        # poison the target before the late bytes are queued (and before this call returns): a
        # consumer with no ordering behind wait() reads the poison, never stale bytes of an earlier
        # (correct) proof that the caching allocator handed back in `t`
        t.fill_(0x05)
        torch.cuda.current_stream().synchronize()
        self.side.wait_event(done)
        with torch.cuda.stream(self.side):
            torch.cuda._sleep(self.delay)
            t.copy_(staged)
        t.record_stream(self.side)
        ev = torch.cuda.Event()
        ev.record(self.side)
        return _Work(ev)

    def recv(self, t, src, group=None):
        raise AssertionError("the device branch must not take the host-memory receive")


def split_proof(hip, n, polys, chal, rnd, zh, pts, world, comm=None):
    """One strong-scaled proof through plonkhip.dist.split_proof_step's DEVICE branch
    (via_host=False), every rank a prover of its own on this GPU, helpers stepped first (their
    sends precede rank 0's receives, as on a real node where they run concurrently).  Returns
    (rank 0's proof, the single-prover proof of the same inputs)."""
    from plonkhip.dist import split_proof_step
    comm = comm or NcclSemantics()
    dev = [torch.from_numpy(p).to("cuda") for p in polys]
    provers = [hip.Prover(n, zh, pts) for _ in range(world)]
    try:
        cb = {c: provers[0].chain_bytes(c) for c in (hip.PLK_CHAIN_T2, hip.PLK_CHAIN_T3)}
        bufs = [{c: torch.zeros(b, dtype=torch.uint8, device="cuda") for c, b in cb.items()} for _ in range(world)]
        stream = torch.cuda.current_stream()
        for p in provers:                      # every prover's stream used once (module docstring)
            p.rounds_dev(dev, chal, rnd)
        torch.cuda.synchronize()
        for r in range(1, world):
            torch.cuda._sleep(comm.delay)       # (see the module docstring)
            split_proof_step(provers[r], dev, chal, rnd, bufs[r], r, world, stream, via_host=False, comm=comm)
        got = split_proof_step(provers[0], dev, chal, rnd, bufs[0], 0, world, stream, via_host=False, comm=comm)
        torch.cuda.synchronize()
        want = provers[0].rounds_dev(dev, chal, rnd)
        return got, want
    finally:
        torch.cuda.synchronize()
        for p in provers:
            p.close()
