"""Breakdown of bench.py's timed region on one GPU (lab tool): the launch loop, the
records -> partials step, the finish (its nonzero() is the host's wait for the device) and the
final synchronize, for 4 consecutive timed regions of K = 20 steps of B MSMs (B from $B, default
40).  The first region of a process was ~0.13 ms slower than the rest (clocks after an idle gap).

    B=160 python tools/timing_probe.py
"""
import sys, time, os, json
sys.path.insert(0, "."); sys.path.insert(0, "plonk.c_amd")
import torch, plonkhip as hip
from plonkhip.dist import finish_sharded, gpu_ops
import bench
hip.init(0); dev = torch.device("cuda", 0); st = torch.cuda.current_stream()
n = 1 << 22; B = int(os.environ.get("B", "40")); K = 20; W = 5
sets = 2 * B if B >= 40 else 80
pts, sc = bench.make_shard_sets(torch, n, 0, n, sets, dev, lambda s: 1234 + s)
ops = gpu_ops(hip, st)
res = torch.zeros(((W + K) * B, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
def launch(first, count):
    i = first
    while i < first + count:
        b = min(B, first + count - i, sets - i % sets); s0 = i % sets
        ops.launch(pts[s0], 3 * n, sc[s0], n, n, b, res[i:]); i += b
for rep in range(4):
    launch(0, W * B)
    finish_sharded(ops.records_to_partials(res[:W * B]), n, ops, lambda j: (pts[j % sets], sc[j % sets]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launch(W * B, K * B)
    t1 = time.perf_counter()
    e = torch.cuda.Event(); e.record(st)
    partials = ops.records_to_partials(res[W * B:])
    t2 = time.perf_counter()
    g1t, folded = finish_sharded(partials, n, ops, None)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    e2 = torch.cuda.Event(); e2.record(st); torch.cuda.synchronize()
    print(json.dumps({"B": B, "launch_loop_ms": round((t1-t0)*1e3,3), "r2p_ms": round((t2-t1)*1e3,3), "finish_ms": round((t3-t2)*1e3,3), "sync_ms": round((t4-t3)*1e3,3), "total_ms": round((t4-t0)*1e3,3)}), flush=True)
