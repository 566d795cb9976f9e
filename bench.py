#!/usr/bin/env python3
"""Benchmark of the PLONK hot path on MI355X (BASELINE.json metric).

Headline (`value`): G1-MSM Mpoint/s -- the KZG commitment MSM srs_eval_at_s
(reference src/srs.h:53-68) over 2^22-point MSMs (config "2^22-point G1 MSM"), inputs resident
in HBM, rotated over > 512 MiB of distinct input sets so no step is served from the 256 MiB
Infinity Cache.  A step = one batched launch of --msm-batch complete MSMs (3 B point + 1 B scalar
per point) finished to G1s.

Multi-GPU (one process per GPU, torch.distributed over RCCL): by default STRONG scaling, the
config SURVEY §8 d3 names -- every 2^22-point MSM is split into contiguous point ranges
(plonkhip.dist.shard_range), rank r reads only its range, and the partial discrete logs of all
K steps are finished by plonkhip.dist.finish_sharded: ONE RCCL all-reduce SUM + the log -> point
map (+ the gathered serial fold for MSMs with irregular encodings).  --weak: every rank owns a
2^22-point shard of an N * 2^22-point MSM instead.  After timing, rank 0 recomputes the first
MSM on one GPU and (strong, 2^22) the sharded path runs the reference golden input
tests/golden/msm.json large[7]; both results are reported.

Also reported (rank 0, `components`): one 2^22 MSM per launch, the 2^16-point MSM (config C2),
the 2^20 forward NTT (config C3) and poly_mul 2^19 x 2^19 with their rooflines, the 2^20-gate
prove (C5: plain, preprocessed, and the pieces of its strong-scaled form; at N > 1 replicas on
every GPU and one proof strong-scaled over up to 3 GPUs), and the reference CPU path timed on this
host (MSM, schoolbook poly_mul, toy prove).

    python bench.py [--gpus N --steps K --warmup W --log2n 22 --weak]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)
MSM_BYTES_PER_POINT = 4  # 3 B G1 + 1 B HF read once
NTT_BYTES_PER_ELEM = 8   # u32 read + write once
# the MSM kernel's translation unit and every header it includes (tests/test_lint_cpu.py checks the
# list against the #include lines): a committed PMC record is valid only for these bytes
MSM_SOURCES = ("msm.hip", "plk_device.h", "plk_internal.h", "plk_msm_finish.h")


def roofline_obj(alg_bytes, ms, what):
    """HBM roofline of a component: algorithmic bytes / measured device time vs the spec peak"""
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "alg_bytes": int(alg_bytes), "alg_bytes_def": what}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks, one process per GPU).  Under a launcher (WORLD_SIZE set) it must equal "
                         "WORLD_SIZE; without one, N > 1 starts `python -m torch.distributed.run --nproc-per-node N` "
                         "on this script as a child process and exits with its status")
    ap.add_argument("--steps", type=int, default=200,
                    help="timed steps; a step is ONE batched launch of --msm-batch MSMs over distinct input sets")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2n", type=int, default=22)
    ap.add_argument("--msm-batch", type=int, default=160,
                    help="MSMs per step = per kernel launch (plk_msm_g1_batch_dev).  160: at N = 8 (strong) a "
                         "rank's share of a step is 160 x 2^19 points = 320 MiB (~55 us of streaming), so the "
                         "timed region's fixed cost (~0.23 ms: first launch, finish, synchronize, the collective) "
                         "stays a few %% of K = 20 steps; with 40 it was 11 %% even at N = 1")
    ap.add_argument("--rotate-mib", type=int, default=640)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-components", action="store_true", help="same as --components none")
    ap.add_argument("--components", default="all",
                    help="all | none | comma list of: msm, ntt, polymul, polyops, prove, cpu -- what rank 0 "
                         "reports beside the headline; at N > 1 'prove' (in 'all') runs C5's replica leg "
                         "(one concurrent proof per GPU) and its strong-scaled leg (one proof over up to 3 GPUs)")
    ap.add_argument("--profile-only", action="store_true",
                    help="just launch the timed MSM loop (for rocprofv3 runs)")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: every rank owns a full 2^log2n-point shard (default: strong, each "
                         "2^log2n-point MSM split over the ranks)")
    return ap.parse_args()


KG16 = [[1, 2, 0], [68, 74, 0], [26, 45, 0], [65, 98, 0], [12, 32, 0], [32, 42, 0], [91, 35, 0], [18, 49, 0],
        [18, 52, 0], [91, 66, 0], [32, 59, 0], [12, 69, 0], [65, 3, 0], [26, 56, 0], [68, 27, 0], [1, 99, 0]]


def make_msm_set(torch, n, dev, seed):
    """One synthetic MSM input: SRS points kG (k uniform in [1,16], G = (1,2)) and HF scalars in
    [0,16], from a device generator seeded per set (any rank can rebuild any set)."""
    kg = torch.tensor(KG16, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    k = torch.randint(0, 16, (n,), generator=g, device=dev)
    pts = kg[k].reshape(-1)
    sc = torch.randint(0, 17, (n,), generator=g, device=dev, dtype=torch.int16).to(torch.uint8)
    return pts, sc


def make_shard_sets(torch, n, lo, hi, sets, dev, seed_of):
    """Rows s = this rank's point range [lo, hi) of input set s (seed seed_of(s))."""
    m = hi - lo
    pts = torch.empty((sets, 3 * m), dtype=torch.uint8, device=dev)
    sc = torch.empty((sets, m), dtype=torch.uint8, device=dev)
    for s in range(sets):
        p, c = make_msm_set(torch, n, dev, seed_of(s))
        pts[s] = p[3 * lo:3 * hi]
        sc[s] = c[lo:hi]
    return pts, sc


def make_msm_sets(torch, n, sets, dev, seed):
    """`sets` full n-point inputs (rows), seeds seed + s."""
    return make_shard_sets(torch, n, 0, n, sets, dev, lambda s: seed + s)


def event_avg_ms(torch, st, fn, reps, rounds=3):
    """Device time per call of fn(i): one event pair around `reps` back-to-back calls on st.
    One call is enqueued BEFORE the start event, so the device is already busy when the
    timed region opens (otherwise the host-side launch latency of the first call is
    counted); a pair per call would add its own ~6 us each.  Returns (best, median) over
    `rounds` rounds."""
    per = []
    for r in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn(r * (reps + 1))
        e0.record(st)
        for i in range(reps):
            fn(r * (reps + 1) + 1 + i)
        e1.record(st)
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) / reps)
    per.sort()
    return per[0], per[len(per) // 2]


def graph_avg_ms(torch, fn, reps, rounds=3):
    """Device time per call of fn(i, stream) with the host out of the loop: `reps` calls
    captured once into a HIP graph (the library's launches go to the capture stream), the graph
    replayed between an event pair.  Short kernels launched one Python call at a time are
    host-rate bound (the ctypes call + hipLaunchKernel ~6 us); replayed they run back to back
    with only the dependent-launch boundary between them.  Returns (best, median) or None when
    capture is not possible."""
    try:
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            fn(0, cs)                            # warm (lazy init outside the capture)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
            for i in range(reps):
                fn(i, cs)
        torch.cuda.synchronize()
    except Exception:
        return None
    per = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(cs):
            e0.record(cs)
            g.replay()
            e1.record(cs)
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) / reps)
    per.sort()
    return per[0], per[len(per) // 2]


def cpu_baseline(pts_np, sc_np, budget_s, gpu_g1):
    """Reference CPU MSM (oracle/_ref = the unmodified reference srs_eval_at_s, -O2) on this
    host, 1 thread.  No silent substitute: without the reference build the baseline is an
    error entry (and main() records a failed check), never a timing of the restatement."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Reference
    if not Reference.available():
        return {"error": "oracle/_ref/libplonkref.so is absent (built by `make -C oracle` where /root/reference "
                         "exists; it travels with the tree): the reference CPU baseline was not measured",
                "kind": "reference", "value": None}
    impl, kind = Reference(), "reference"
    t0 = time.perf_counter()
    out = impl.msm(pts_np, sc_np)
    dt = time.perf_counter() - t0
    reps = 1
    while time.perf_counter() - t0 < budget_s:
        impl.msm(pts_np, sc_np)
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    n = sc_np.size
    return {"value": round(n / dt / 1e6, 3), "unit": "Mpoint/s", "cores": 1, "kind": kind,
            "sample": "srs_eval_at_s over the first timed input set (%d points, subgroup points, "
                      "scalars in [0,16]), %d repetitions, gcc -O2, single thread" % (n, reps),
            "seconds_per_msm": round(dt, 4), "matches_gpu": out == gpu_g1}


def kernel_source_hash():
    """SHA-256 (16 hex) of the MSM kernel's sources: a PMC record is used only for this code."""
    import hashlib
    h = hashlib.sha256()
    for f in MSM_SOURCES:
        with open(os.path.join(ROOT, "plonk.c_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(log2n, batch, m):
    """roofline.traffic: HBM bytes per launch from the committed PMC pass
    (profiles/msm_pmc_latest.json, tools/pmc_summary.py), only when it was measured for this
    launch shape AND this kernel source; otherwise None."""
    path = os.path.join(ROOT, "profiles", "msm_pmc_latest.json")
    try:
        with open(path) as f:
            j = json.load(f)
    except (OSError, ValueError):
        return None, "msm_dlog_kernel"
    kname = j.get("kernel", "msm_dlog_kernel").split("(")[0].replace("void ", "")
    ok = (j.get("log2n") == log2n and j.get("msm_batch") == batch and m == 1 << log2n and
          j.get("source_sha16") == kernel_source_hash())
    return (j.get("hbm_bytes_per_launch") if ok else None), kname


def one_msm_log(torch, hip, pts, sc, n, dev, st):
    """discrete log of one MSM over a full input (single GPU)"""
    rec = torch.zeros(hip.MSM_RESULT_BYTES, dtype=torch.uint8, device=dev)
    hip.msm_g1_dev(pts, sc, n, rec, st)
    torch.cuda.synchronize()
    return int(rec[hip.MSM_LOG_OFFSET:hip.MSM_LOG_OFFSET + 4].view(torch.int32).item())


def single_msm_component(torch, hip, pts, sc, m, sets, dev):
    """ONE m-point MSM per launch (the literal north-star case), launches back to back from a
    HIP graph (host out of the loop), cold input sets; frac against the HBM spec peak."""
    r1 = torch.zeros((64, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
    gr = graph_avg_ms(torch, lambda i, s: hip.msm_g1_dev(pts[i % sets], sc[i % sets], m, r1[i % 64], s), 64)
    if gr is None:
        st = torch.cuda.current_stream()
        gr = event_avg_ms(torch, st, lambda i: hip.msm_g1_dev(pts[i % sets], sc[i % sets], m, r1[i % 64], st), 64)
    avg, med = gr
    gbs = MSM_BYTES_PER_POINT * m / (avg * 1e-3) / 1e9
    return {"device_us_per_msm": round(avg * 1e3, 2), "median_us": round(med * 1e3, 2),
            "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "alg_bytes": MSM_BYTES_PER_POINT * m,
            "note": "unbatched: one launch per MSM, 64 launches replayed back to back as a HIP graph (includes "
                    "the dependent-launch boundary); rocprofv3 kernel duration in profiles/"}


def cpu_other_baselines(hip):
    """The reference's other hot paths on this host (oracle/_ref: the unmodified reference
    headers, gcc -O2, one thread), bounded samples: schoolbook poly_mul (src/poly.h:106-122) at
    2^14 x 2^14 and 2^15 x 2^15 with the O(la lb) extrapolation to config C3's 2^19 x 2^19, and the
    toy prove of src/plonk-test.c (src/plonk.h:223) next to the same proof through the drop-in
    build: as shipped (toy-size calls on the host, include/plk_host.h) and with every call on the GPU."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gen
    from pyoracle import Reference
    if not Reference.available():
        return {"note": "oracle/_ref absent on this host"}
    R = Reference()
    out = {}
    for k in (14, 15):
        a, b = gen.poly_inputs(0xC0DE + k, 1 << k, 1 << k)
        t0 = time.perf_counter()
        R.poly_mul(a, b)
        dt = time.perf_counter() - t0
        out["poly_mul_2^%dx2^%d" % (k, k)] = {"s": round(dt, 4), "GMAC_s": round((1 << 2 * k) / dt / 1e9, 3)}
    rate = out["poly_mul_2^15x2^15"]["GMAC_s"] * 1e9
    out["poly_mul_2^19x2^19_extrapolated_s"] = round((1 << 38) / rate, 1)
    with open(os.path.join(ROOT, "tests", "golden", "prove.json")) as f:
        p = json.load(f)["proofs"][0]
    args = (p["gates"], p["copies"], p["wires"], p["chal"], p["rand"], p["secret"], p["srs_n"], p["srs_mode"])
    reps = 20000
    t0 = time.perf_counter()
    for _ in range(reps):
        proof = R.prove4_inproc(*args)
    ref_us = (time.perf_counter() - t0) / reps * 1e6
    out["toy_prove_4_gates"] = {"reference_cpu_us": round(ref_us, 2), "matches_golden": proof.hex() == p["proof"]}
    dropin = os.path.join(ROOT, "oracle", "_ref", "libplonkref_dropin.so")
    if os.path.exists(dropin):
        D = Reference(dropin)
        toy = out["toy_prove_4_gates"]

        def timed(n):
            D.prove4_inproc(*args)
            t0 = time.perf_counter()
            for _ in range(n):
                pr = D.prove4_inproc(*args)
            return round((time.perf_counter() - t0) / n * 1e6, 2), pr.hex() == p["proof"]

        # the drop-in as shipped: include/plk_host.h keeps toy-size calls on the host
        toy["dropin_us"], toy["dropin_matches_golden"] = timed(reps)
        toy["dropin_vs_reference_cpu"] = round(toy["dropin_us"] / ref_us, 3)
        # the same build with the policy's threshold at 0: every poly_mul / MSM / division / evaluation /
        # matrix call of the toy prove crosses to the GPU
        with hip.options(DROPIN_HOST_WORK=0):
            toy["dropin_all_gpu_us"], toy["dropin_all_gpu_matches_golden"] = timed(50)
    out["note"] = ("reference compiled from its own headers (oracle/_ref, gcc -O2), 1 thread, in-process; the toy "
                   "prove = srs_create + plonk_new + plonk_prove of src/plonk-test.c; dropin_us: the same program "
                   "built against include/ (libplonkref_dropin.so) with the default small-size policy, which keeps "
                   "its toy-size calls on the host (include/plk_host.h, PLK_OPT_DROPIN_HOST_WORK 32768); "
                   "dropin_all_gpu_us: the policy at 0, every poly_mul / MSM / poly_divide / poly_eval / matrix call "
                   "on the GPU one tiny call at a time (latency-bound: ~100 host<->device round trips)")
    return out


COMPONENT_GROUPS = ("msm", "ntt", "polymul", "polyops", "prove", "cpu")


def wanted_components(args):
    """the set of component groups this run reports"""
    if args.no_components or args.components == "none":
        return set()
    if args.components == "all":
        return set(COMPONENT_GROUPS)
    want = {c.strip() for c in args.components.split(",") if c.strip()}
    bad = want - set(COMPONENT_GROUPS)
    if bad:
        raise SystemExit("unknown --components %s (choose from %s)" % (sorted(bad), ", ".join(COMPONENT_GROUPS)))
    return want


def pts_label(m):
    """component key fragment naming the points one MSM actually reads: 2^k, or the count"""
    return "2^%d" % (m.bit_length() - 1) if m & (m - 1) == 0 else "%dpts" % m


def components(torch, hip, dev, st, want):
    out = {}
    if "msm" in want:
        out.update(msm_components(torch, hip, dev, st))
        out["host_call_msm_2^22_devices"] = msm_host_devices_component(torch, hip, dev)
    if "ntt" in want:
        out.update(ntt_components(torch, hip, dev, st))
    if "polymul" in want:
        out.update(polymul_components(torch, hip, dev, st))
    if "polyops" in want:
        out.update(polyops_components(torch, hip, dev, st))
    if "prove" in want:
        out["prove_2^20_gates"] = prove_component(torch, hip, dev, 20)
        out["prove_2^20_gates_preprocessed"] = prove_component(torch, hip, dev, 20, preprocessed=True)
        out["prove_2^20_gates_split_pieces"] = prove_split_pieces(torch, hip, dev, 20)
        out["prove_2^20_gates_c_split_rehearsal"] = prove_c_split_rehearsal(torch, hip, dev, 20)
    return out


def msm_components(torch, hip, dev, st):
    out = {}
    # C2: 2^16-point MSM -- device-resident kernel time and host-buffer call (PCIe incl.)
    n = 1 << 16
    pts, sc = make_msm_sets(torch, n, 8, dev, 7)
    res = torch.zeros((64, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
    eag, _ = event_avg_ms(torch, st, lambda i: hip.msm_g1_dev(pts[i % 8], sc[i % 8], n, res[i % 64], st), 64)
    gr = graph_avg_ms(torch, lambda i, s: hip.msm_g1_dev(pts[i % 8], sc[i % 8], n, res[i % 64], s), 64)
    avg, med = gr if gr else (eag, eag)
    ph, sh = pts[0].cpu().numpy(), sc[0].cpu().numpy()
    hip.msm_g1(ph, sh)
    t0 = time.perf_counter()
    for _ in range(20):
        hip.msm_g1(ph, sh)
    host_us = (time.perf_counter() - t0) / 20 * 1e6
    out["msm_2^16"] = {"device_us_per_msm": round(avg * 1e3, 2), "median_us": round(med * 1e3, 2),
                       "Mpoint_s": round(n / (avg * 1e-3) / 1e6, 1),
                       "eager_us_per_call": round(eag * 1e3, 2),
                       "host_call_us_incl_pcie": round(host_us, 1),
                       "note": "one launch per MSM, back-to-back on one stream: device time from 64 launches "
                               "replayed as a HIP graph%s; eager_us_per_call = one Python call per launch "
                               "(host-rate bound)" % ("" if gr else " (capture unavailable: eager)")}
    # the drop-in's srs_eval_at_s path (plk_msm_g1, host buffers): 2^20 points, the SRS bytes
    # unchanged between calls (device copy reused after a memcmp) vs a fresh SRS array each call
    n20 = 1 << 20
    p20, s20 = make_msm_sets(torch, n20, 1, dev, 99)
    ph20, sh20 = p20[0].cpu().numpy(), s20[0].cpu().numpy()
    hip.msm_g1(ph20, sh20)
    t0 = time.perf_counter()
    for _ in range(10):
        hip.msm_g1(ph20, sh20)
    cached_us = (time.perf_counter() - t0) / 10 * 1e6
    copies = [ph20.copy() for _ in range(10)]
    t0 = time.perf_counter()
    for c in copies:
        hip.msm_g1(c, sh20)
    fresh_us = (time.perf_counter() - t0) / 10 * 1e6
    out["msm_2^20_host_call"] = {"srs_cached_us": round(cached_us, 1), "srs_uploaded_us": round(fresh_us, 1),
                                 "note": "plk_msm_g1 (what the drop-in srs_eval_at_s calls), host buffers, PCIe "
                                         "included; cached = same SRS pointer and bytes (reference: 9 commitments "
                                         "per proof over one SRS, src/plonk.h:299-301,379,522-524,620-621)"}
    return out


def msm_host_devices_component(torch, hip, dev, n=1 << 22):
    """srs_eval_at_s's host-buffer call (plk_msm_g1, PCIe included) at 2^22 points on one device
    and split over several (plk_init_devices: per-device uploads from per-shard host threads, host
    sum of the partial logs).  On a one-GPU box the list repeats device 0 (the N-device code path,
    one device's link); on a multi-GPU node `all_devices` also names every visible GPU (measured in a
    child process, tools/devices_probe.py, so that a multi-device failure cannot cost the line)."""
    import numpy as np
    ndev = torch.cuda.device_count()
    lists = [[0], [0, 0], [0, 0, 0, 0]]   # (distinct devices: a child process below)
    p, c = make_msm_sets(torch, n, 1, dev, 4242)
    ph, sh = p[0].cpu().numpy(), c[0].cpu().numpy()
    out = {"points": n, "note": "plk_msm_g1 wall time per call from host buffers; cached = same SRS pointer and "
                                "bytes (memcmp-verified per shard), uploaded = a fresh SRS array each call; "
                                "lists of one repeated device rehearse the multi-device path on one GPU"}
    want = None
    try:
        for ids in lists:
            hip.init_devices(ids)
            got = hip.msm_g1(ph, sh)
            want = want or got
            ok = True
            cached, fresh = [], []
            for _ in range(3):          # best / median of 3 rounds (host timings are noisy)
                t0 = time.perf_counter()
                for _ in range(5):
                    ok &= hip.msm_g1(ph, sh) == want
                cached.append((time.perf_counter() - t0) / 5 * 1e6)
                copies = [ph.copy() for _ in range(3)]    # (written: their pages exist before timing)
                t0 = time.perf_counter()
                for cp in copies:
                    ok &= hip.msm_g1(cp, sh) == want
                fresh.append((time.perf_counter() - t0) / 3 * 1e6)
            cached.sort()
            fresh.sort()
            out["devices_" + "_".join(map(str, ids))] = {"srs_cached_us": round(cached[0], 1),
                                                         "srs_cached_median_us": round(cached[1], 1),
                                                         "srs_uploaded_us": round(fresh[0], 1),
                                                         "srs_uploaded_median_us": round(fresh[1], 1),
                                                         "same_result": bool(ok and got == want)}
    finally:
        hip.init_devices([0])
    if ndev > 1:
        # every visible GPU through plk_init_devices, in a child process with its own contexts and a
        # time limit (a multi-device failure must not cost this line)
        import subprocess
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "devices_probe.py")], capture_output=True,
                               text=True, timeout=240)
            lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
            out["all_devices"] = json.loads(lines[-1]) if r.returncode == 0 and lines else {
                "error": "exit %d: %s" % (r.returncode, r.stderr.strip()[-300:])}
        except subprocess.TimeoutExpired:
            out["all_devices"] = {"error": "timed out after 240 s"}
    return out


def ntt_components(torch, hip, dev, st):
    out = {}
    nb = 8
    # C3: forward NTT 2^20 over BabyBear (Montgomery u32, in place, 2 passes)
    k = 20
    bufs = [torch.randint(0, 2013265921, (1 << k,), dtype=torch.int64, device=dev).to(torch.int32)
            for _ in range(4)]
    for b in bufs:
        hip.ntt_dev(b, k, False, st)
    eag, _ = event_avg_ms(torch, st, lambda i: hip.ntt_dev(bufs[i % 4], k, False, st), 50)
    gr = graph_avg_ms(torch, lambda i, s: hip.ntt_dev(bufs[i % 4], k, False, s), 50)
    avg, med = gr if gr else (eag, eag)
    alg = NTT_BYTES_PER_ELEM * (1 << k)
    out["ntt_2^20_forward"] = {"ms": round(avg, 4), "eager_ms": round(eag, 4),
                               "Gelem_s": round((1 << k) / (avg * 1e-3) / 1e9, 2), "passes": 2,
                               "roofline": roofline_obj(alg, avg, "SURVEY 8(d): u32 read + write once per element"),
                               "inputs": "4 rotating 4 MiB arrays: Infinity-Cache resident, as when a transform follows "
                                         "the kernel that wrote its input; ms_cold: 136 arrays (544 MiB, twice the cache) rotated"}
    # the same with cold inputs (SURVEY 8(d) cache caveat): 136 arrays (544 MiB > 2 x the 256 MiB
    # Infinity Cache) rotated, every launch of a replay on a different array
    ncold = 136
    cold = torch.empty((ncold, 1 << k), dtype=torch.int32, device=dev)
    cold.random_(0, 2013265921)
    gr = graph_avg_ms(torch, lambda i, s: hip.ntt_dev(cold[i % ncold], k, False, s), ncold)
    if gr:
        out["ntt_2^20_forward"]["ms_cold"] = round(gr[1], 4)
    del cold
    # the same transform, 8 independent arrays sharing each pass's launch (plk_ntt_batch_dev)
    bb_ = [torch.randint(0, 2013265921, (nb, 1 << k), dtype=torch.int64, device=dev).to(torch.int32)
           for _ in range(2)]
    gr = graph_avg_ms(torch, lambda i, s: hip.ntt_batch_dev(bb_[i % 2], k, nb, False, s), 20)
    avg, med = gr if gr else event_avg_ms(torch, st, lambda i: hip.ntt_batch_dev(bb_[i % 2], k, nb, False, st), 20)
    out["ntt_2^20_forward_batch8"] = {"ms_per_launch": round(avg, 4),
                                      "Gelem_s": round(nb * (1 << k) / (avg * 1e-3) / 1e9, 2),
                                      "roofline": roofline_obj(nb * alg, avg, "8 transforms per launch")}
    # C3 in the field poly_mul and the prover transform in: F29 (plk_ntt29_dev, lazy reduction,
    # fully reduced outputs), single and 8 per launch
    P29 = 7 * (1 << 26) + 1
    b29 = [torch.randint(0, P29, (1 << k,), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(4)]
    for b in b29:
        hip.ntt29_dev(b, k, False, st)
    gr = graph_avg_ms(torch, lambda i, s: hip.ntt29_dev(b29[i % 4], k, False, s), 50)
    avg, med = gr if gr else event_avg_ms(torch, st, lambda i: hip.ntt29_dev(b29[i % 4], k, False, st), 50)
    out["ntt29_2^20_forward"] = {"ms": round(avg, 4), "Gelem_s": round((1 << k) / (avg * 1e-3) / 1e9, 2),
                                 "passes": 2,
                                 "roofline": roofline_obj(alg, avg, "SURVEY 8(d): u32 read + write once per element")}
    b29 = [torch.randint(0, P29, (nb, 1 << k), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(2)]
    gr = graph_avg_ms(torch, lambda i, s: hip.ntt29_batch_dev(b29[i % 2], k, nb, False, s), 20)
    avg, med = gr if gr else event_avg_ms(torch, st, lambda i: hip.ntt29_batch_dev(b29[i % 2], k, nb, False, st), 20)
    out["ntt29_2^20_forward_batch8"] = {"ms_per_launch": round(avg, 4),
                                        "Gelem_s": round(nb * (1 << k) / (avg * 1e-3) / 1e9, 2),
                                        "roofline": roofline_obj(nb * alg, avg, "8 transforms per launch")}
    del b29
    for key, peak, nt in (("ntt_2^20_forward", "bb_dif_Gbfly_s", 1), ("ntt_2^20_forward_batch8", "bb_dif_Gbfly_s", 8),
                          ("ntt29_2^20_forward", "f29_dif_Gbfly_s", 1),
                          ("ntt29_2^20_forward_batch8", "f29_dif_Gbfly_s", 8)):
        c = out[key]
        bfly = butterfly_roofline(nt * (1 << 19) * 20, c.get("ms", c.get("ms_per_launch")), peak)
        if bfly:
            c["roofline_butterfly"] = bfly
    return out


def polymul_components(torch, hip, dev, st):
    out = {}
    # poly_mul 2^19 x 2^19 -> 2^20 - 1 coefficients (device-resident)
    la = lb = 1 << 19
    a = torch.randint(0, 17, (la,), dtype=torch.int16, device=dev).to(torch.uint8)
    b = torch.randint(0, 17, (lb,), dtype=torch.int16, device=dev).to(torch.uint8)
    o = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
    nz = torch.zeros(4, dtype=torch.int32, device=dev)
    work = torch.zeros(hip.poly_mul_workspace(la, lb), dtype=torch.uint8, device=dev)
    hip.poly_mul_dev(a, la, b, lb, o, nz, work, st)
    gr = graph_avg_ms(torch, lambda i, s: hip.poly_mul_dev(a, la, b, lb, o, nz, work, s), 30)
    avg, med = gr if gr else event_avg_ms(torch, st, lambda i: hip.poly_mul_dev(a, la, b, lb, o, nz, work, st), 30)
    out["poly_mul_2^19x2^19"] = {"ms": round(avg, 4), "Gcoeff_s_out": round((la + lb - 1) / (avg * 1e-3) / 1e9, 2),
                                 "roofline": roofline_obj(la + lb + (la + lb - 1), avg,
                                                          "SURVEY 8(d): la + lb + (la + lb - 1) bytes of HF")}
    # three 2^20-point transforms over F29 (a and b forward, the product inverse): 3 x 2^19 x 20
    # butterflies
    bfly = butterfly_roofline(3 * (1 << 19) * 20, avg, "f29_dif_Gbfly_s",
                              mix=[("f29_dif", 2 / 3), ("f29_dit", 1 / 3)])
    if bfly:
        out["poly_mul_2^19x2^19"]["roofline_butterfly"] = bfly
    return out


# Integer-VALU instruction mix of one radix-2 butterfly as the engine compiles it (ntt_wave.hip
# F29 / FBB policies, plk_device.h primitives; counted in the gfx950 ISA): v_mad_u64_u32 and
# 32-bit VALU ops (add / sub / min / mul_lo).  Issue rates measured by tools/isa_clock.hip at
# 8 waves per SIMD: 4.5 cycles per v_mad_u64_u32 and 4.2 per 32-bit op per wave-instruction.
ISA_BFLY = {"f29_dif": (3, 3), "f29_dit": (2, 5), "bb_dif": (2, 8), "bb_dit": (2, 9)}
ISA_CYC = (4.5, 4.2)
CU_SIMDS, CLOCK_HZ = 1024, 2.4e9   # 256 CUs x 4 SIMDs; MI355X peak engine clock (MI355X_MICROARCH.md)


def isa_bound_gbfly(kind):
    """hardware bound: every SIMD issuing the butterfly's instruction mix back to back"""
    mads, ops = ISA_BFLY[kind]
    cyc = mads * ISA_CYC[0] + ops * ISA_CYC[1]
    return CU_SIMDS * 64 * CLOCK_HZ / cyc / 1e9


def butterfly_roofline(bfly, ms, key, mix=None):
    """Compute roofline of an NTT component: radix-2 butterflies / time against (a) the butterfly
    peak measured by tools/bfly_peak.hip (the engine's own formulas in registers, no memory;
    committed in profiles/r02_bfly_peak.json -- a peak, like the HBM spec peak, not a timing of
    this run) and (b) the ISA bound of the same butterflies (isa_bound_gbfly; mix = [(kind,
    share)] for a product's forward DIF + inverse DIT transforms)."""
    try:
        with open(os.path.join(ROOT, "profiles", "r02_bfly_peak.json")) as f:
            pk = json.loads([l for l in f if l.startswith("{")][0])
    except (OSError, IndexError, ValueError):
        return None
    rate = bfly / (ms * 1e-3) / 1e9
    mix = mix or [({"f29_dif_Gbfly_s": "f29_dif", "bb_dif_Gbfly_s": "bb_dif"}[key], 1.0)]
    # time-weighted: a share s of the butterflies at bound b costs s / b
    isa = 1.0 / sum(sh / isa_bound_gbfly(kind) for kind, sh in mix)
    return {"bound": "valu", "achieved": round(rate, 1), "peak": pk[key], "unit": "Gbutterfly/s",
            "frac": round(rate / pk[key], 4), "butterflies": int(bfly),
            "isa_bound": round(isa, 1), "frac_of_isa_bound": round(rate / isa, 4),
            "isa_mix": {k: {"v_mad_u64_u32": ISA_BFLY[k][0], "valu32": ISA_BFLY[k][1], "share": sh} for k, sh in mix},
            "peak_source": "profiles/r02_bfly_peak.json (%s); isa_bound: instruction mix x tools/isa_clock.hip issue "
                           "rates x 1024 SIMDs x 2.4 GHz" % key}


def polyops_components(torch, hip, dev, st):
    """SURVEY 8 (f) rows at the boundary, device-resident: poly_divide by Z_H = x^n - 1
    (src/poly.h:124-177; the prover's t(x) division, n = 2^20, numerator 4n) and a batch of 8
    poly_eval over 2^22-coefficient polynomials (src/poly.h:265-272); both read their inputs once,
    so the HBM roofline applies (canonical random coefficients)."""
    import numpy as np
    out = {}
    n = 1 << 20
    nl = 4 * n
    num = torch.randint(0, 17, (nl,), dtype=torch.int16, device=dev).to(torch.uint8)
    den = np.zeros(n + 1, np.uint8)
    den[0], den[n] = 16, 1
    quot = torch.zeros(nl, dtype=torch.uint8, device=dev)
    rem = torch.zeros(n, dtype=torch.uint8, device=dev)
    lens = torch.zeros(4, dtype=torch.int32, device=dev)
    work = torch.zeros(max(16, hip.poly_divide_workspace(nl, n + 1)), dtype=torch.uint8, device=dev)
    call = lambda i, s: hip.poly_divide_dev(num, nl, den, quot, rem, lens, work, s)   # noqa: E731
    gr = graph_avg_ms(torch, call, 20)
    avg, _ = gr if gr else event_avg_ms(torch, st, lambda i: call(i, st), 20)
    alg = nl + (nl - n) + n    # numerator read once, quotient and remainder written once
    out["poly_divide_zh_2^22"] = {"ms": round(avg, 4), "roofline": roofline_obj(alg, avg,
                                  "numerator read + quotient and remainder written once (bytes of HF)"),
                                  "note": "plk_poly_divide_dev by x^(2^20) - 1, numerator 2^22 coefficients"}
    m = 8
    polys = [torch.randint(0, 17, (nl,), dtype=torch.int16, device=dev).to(torch.uint8) for _ in range(m)]
    ys = torch.zeros(m, dtype=torch.uint8, device=dev)
    tick = torch.zeros(max(16, hip.poly_eval_workspace(m)), dtype=torch.uint8, device=dev)
    xs = np.arange(2, 2 + m, dtype=np.uint8)
    call = lambda i, s: hip.poly_eval_batch_dev(polys, [nl] * m, xs, ys, tick, s)   # noqa: E731
    gr = graph_avg_ms(torch, call, 20)
    avg, _ = gr if gr else event_avg_ms(torch, st, lambda i: call(i, st), 20)
    out["poly_eval_batch8_2^22"] = {"ms": round(avg, 4), "roofline": roofline_obj(m * nl, avg,
                                    "every coefficient byte read once"),
                                    "note": "plk_poly_eval_batch_dev: 8 polynomials of 2^22 coefficients per launch"}
    return out


def _prove_golden(n, out):
    """True / False against tests/golden/prove_2_20.json when it holds this size, else None"""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "prove_2_20.json")) as f:
            g = json.load(f)
    except OSError:
        return None
    return out.hex() == g["proof"] if g["n"] == n and g["seed"] == 51 else None


def prove_component(torch, hip, dev, log2n, reps=9, preprocessed=False, barrier=None):
    """C5: plonk_prove rounds 1-5 (src/plonk.h:277-655) at n = 2^log2n gates on the device
    prover: 17 poly_mul (largest (3n+4) x (n+3) -> NTT 2^(log2n+3)), 9 commitments, 3
    divisions, evaluations.  Synthetic interpolated polynomials (GF(17) has no subgroup of
    order 2^20, so no satisfiable circuit exists at this size) and a random SRS long enough
    for every commitment; non-strict (remainders not asserted).  Wall time per call, the
    call synchronous and returning the 34 proof bytes to the host.  preprocessed: the six fixed
    circuit polynomials' round-3 transforms computed once beforehand (plk_prover_preprocess,
    outside the timed calls -- PLONK's preprocessed input), every timed call the same proof.
    barrier: called right before the timed calls (the N-GPU replica leg starts every rank's
    proofs together)."""
    n = 1 << log2n
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gen
    # the instance of tests/golden/prove_2_20.json (seed 51, SRS len 2n+8): at n = 2^20 the
    # measured proof is compared with the CPU restatement's recorded answer
    srs_len = 2 * n + 8
    hpolys, chal, rnd, zh, pts = gen.prove_instance(n, 51, srs_len)
    polys = [torch.from_numpy(p).to(dev) for p in hpolys]
    pr = hip.Prover(n, zh, pts)
    first = pr.rounds_dev(polys, chal, rnd)
    pre_ms = None
    if preprocessed:
        t0 = time.perf_counter()
        pr.preprocess(polys)
        pre_ms = round((time.perf_counter() - t0) * 1e3, 3)
        first = pr.rounds_dev(polys, chal, rnd, preprocessed=True)
    torch.cuda.synchronize()
    # the roofline's profiled proofs first: the timed calls (and a profiler's last traced proof) stay
    # plain rounds_dev calls with no events between their launches
    roof, launches = prove_roofline(hip, pr, polys, chal, rnd, preprocessed, first)
    if barrier is not None:
        barrier()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = pr.rounds_dev(polys, chal, rnd, preprocessed=preprocessed)
        t.append(time.perf_counter() - t0)
    t.sort()
    wall = t[len(t) // 2]
    roof["hbm"].update(achieved=round(roof["hbm"]["alg_bytes"] / wall / 1e9, 1),
                       frac=round(roof["hbm"]["alg_bytes"] / wall / 1e9 / HBM_PEAK_GBS, 5))
    extra = {"preprocess_ms_once": pre_ms,
             "preprocessed": "the forward transforms of the six fixed circuit polynomials q_o q_m q_l q_r s_sigma_3 "
                             "l_1_x (PLONK's preprocessed input) computed once by plk_prover_preprocess before the "
                             "timed calls; everything that depends on the witness, blinding or challenges runs in "
                             "every call, and the proof bytes are the same as without"} if preprocessed else {}
    # ms = the MEDIAN of the synchronous calls (the honest figure for one call; box-to-box spread
    # ~3 %); best_ms beside it
    return {"ms": round(t[len(t) // 2] * 1e3, 3), "median_ms": round(t[len(t) // 2] * 1e3, 3),
            "best_ms": round(t[0] * 1e3, 3), "calls": reps, "gates": n, "launches": launches, "roofline": roof, **extra,
            "deterministic": out == first, "matches_oracle": _prove_golden(n, out),
            "device_mib": round(pr.device_bytes() / 2**20, 1),
            "note": "rounds 1-5 of plonk_prove, synthetic interpolated polys (gen.prove_instance, seed 51), SRS len 2n+8, "
                    "host wall time per synchronous call (proof bytes back on the host); matches_oracle: equal to the "
                    "recorded answer of the CPU restatement oracle/prove_ref.py (tests/golden/prove_2_20.json), which is "
                    "pinned to the reference's own proofs at n = 4 -- the reference cannot prove above 4 gates "
                    "(no 2^20-point domain in GF(17)), so parity at 2^20 is pinned through that restatement"}


def prove_roofline(hip, pr, polys, chal, rnd, preprocessed, want, reps=7):
    """C5's roofline for the line.  The proof's NTT kernels -- every pass of round
    3's two product batches -- timed by hipEvents on the prover's own stream around each batch
    (plk_prover_profile_dev, median of `reps` proofs; the span includes the boundaries between the
    batch's launches, so the fraction is a lower bound), their radix-2 butterflies counted from the
    library's launch plan (plk_ntt_launch_log) and priced against the butterfly peaks of
    profiles/r02_bfly_peak.json exactly as tools/ntt_roofline.py prices rocprof durations
    (plonkhip.roofline); the proof's algorithmic bytes (SURVEY 8(d) terms, plk_prover_alg_bytes) over
    the median wall time against the HBM spec peak (filled in by the caller after its timed calls);
    launches = kernel nodes of the call captured as a HIP graph (plk_prover_launches: counted, never
    run).  Returns (roofline dict, launches)."""
    from plonkhip import roofline as RL
    hip.ntt_launch_log()                             # (drop older records)
    with hip.options(NTT_LAUNCH_LOG=1):
        got, _ = pr.profile_dev(polys, chal, rnd, preprocessed)
    plan = hip.ntt_launch_log()
    prof = sorted((pr.profile_dev(polys, chal, rnd, preprocessed) for _ in range(reps)), key=lambda x: x[1]["ntt_ms"])
    med = prof[len(prof) // 2][1]
    same = got == want and all(o == want for o, _ in prof)
    pk = RL.load_peaks(RL.PEAKS)
    tot = RL.plan_roofline(plan, pk)
    kernels, other = pr.launches(polys, chal, rnd, preprocessed)
    alg = pr.alg_bytes()
    ntt_ms = med["ntt_ms"]
    rate = tot["butterflies"] / (ntt_ms * 1e-3)
    roof_ms = tot["roof_s"] * 1e3
    return {"bound": "valu", "unit": "Gbutterfly/s", "achieved": round(rate / 1e9, 1),
            "peak": round(tot["butterflies"] / tot["roof_s"] / 1e9, 1), "frac": round(roof_ms / ntt_ms, 4),
            "butterflies": tot["butterflies"], "roof_ms": round(roof_ms, 4), "ntt_ms": round(ntt_ms, 4),
            "ntt_launches": tot["launches"], "span_ms": round(med["span_ms"], 4),
            "ntt_share_of_span": round(ntt_ms / med["span_ms"], 3),
            "ntt_hbm": {"alg_bytes": tot["bytes"], "frac": round(tot["bytes"] / HBM_PEAK_GBS / 1e9 / (ntt_ms * 1e-3), 4),
                        "def": "8 B per element per pass and array (u32 read + write), 12 B per element per product "
                               "in the centre (DESIGN 4)"},
            "hbm": {"alg_bytes": alg, "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                    "def": "SURVEY 8(d) per-op bytes over the reference's own ops of rounds 1-5 (17 poly_mul, 9 "
                           "srs_eval_at_s, 3 poly_divide, 9 poly_eval; plk_prover_alg_bytes) / the median wall time"},
            "same_proof_while_profiled": same,
            "peak_source": "profiles/r02_bfly_peak.json per launch (forward / shared passes DIF, inverse DIT, centre "
                           "(2 DIF + 1 DIT) / 3, F29 or BabyBear per the launch log); peak = the butterfly-weighted "
                           "harmonic mean",
            "timing": "hipEvents on the prover's stream around round 3's two product batches (plk_prover_profile_dev), "
                      "median of %d proofs" % reps}, kernels


def prove_split_pieces(torch, hip, dev, log2n, reps=5):
    """The pieces of the strong-scaled proof (prove_split_component) timed on this one GPU: rank 0's
    proof with both chains' products already received (plk_prover_rounds_ext_dev, wall time per
    synchronous call) and a helper's chains alone (plk_prover_chains_dev, wall time to the
    products' completion).  With the chains' transfer (4 MiB each over xGMI) hidden behind rank 0's
    own work, rank 0's time is the strong-scaled proof's time: both chains received at 3 GPUs,
    t_3 received at 2."""
    n = 1 << log2n
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gen
    hpolys, chal, rnd, zh, pts = gen.prove_instance(n, 51, 2 * n + 8)
    polys = [torch.from_numpy(p).to(dev) for p in hpolys]
    pr = hip.Prover(n, zh, pts)
    T2, T3 = hip.PLK_CHAIN_T2, hip.PLK_CHAIN_T3
    bufs = {c: torch.zeros(pr.chain_bytes(c), dtype=torch.uint8, device=dev) for c in (T2, T3)}
    single = pr.rounds_dev(polys, chal, rnd)
    pr.chains_dev(polys, chal, rnd, T2 | T3, bufs[T2], bufs[T3])
    torch.cuda.synchronize()

    def best(fn):
        fn()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        return round(min(t) * 1e3, 3)

    def chains(m):
        pr.chains_dev(polys, chal, rnd, m, bufs[T2] if m & T2 else None, bufs[T3] if m & T3 else None)
        torch.cuda.synchronize()

    out = {"single_gpu_ms": best(lambda: pr.rounds_dev(polys, chal, rnd)),
           "rank0_with_chains_received_ms": best(lambda: pr.rounds_ext_dev(polys, chal, rnd, T2 | T3, bufs[T2], bufs[T3])),
           "rank0_with_t3_received_ms": best(lambda: pr.rounds_ext_dev(polys, chal, rnd, T3, None, bufs[T3])),
           "helper_t2_chain_ms": best(lambda: chains(T2)), "helper_t3_chain_ms": best(lambda: chains(T3)),
           "helper_both_chains_ms": best(lambda: chains(T2 | T3)),
           "chain_bytes": pr.chain_bytes(T2),
           "same_proof": pr.rounds_ext_dev(polys, chal, rnd, T2 | T3, bufs[T2], bufs[T3]) == single,
           "note": "one GPU: the strong-scaled proof's pieces (DESIGN 6b); rank0_*: the proving GPU's wall time "
                   "per proof once the chains' products are on it; helper_*: a helper GPU's chain(s) from the "
                   "same inputs, to completion; the multi-GPU time adds the chain products' transfer "
                   "(chain_bytes each) where it is not hidden behind rank 0's own work"}
    pr.close()
    return out


def prove_c_split_rehearsal(torch, hip, dev, log2n, reps=5):
    """The split proof driven from C (plk_prover_attach_helpers over the plk_init_devices list) on
    ONE GPU: lists repeating device 0 put the helper provers on their own streams of the same
    device, so this times the code path and checks its bytes, not a speed-up (the helpers compete
    with the proving prover for the same CUs).  Distinct GPUs: tools/devices_probe.py on
    multi-GPU nodes (components.host_call_msm_2^22_devices.all_devices.prove_2^20_split_from_c)."""
    n = 1 << log2n
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gen
    hpolys, chal, rnd, zh, pts = gen.prove_instance(n, 51, 2 * n + 8)
    polys = [torch.from_numpy(p).to(dev) for p in hpolys]
    pr = hip.Prover(n, zh, pts)
    out = {"note": "one GPU: helpers on their own streams of device 0 (plk_init_devices [0,0] / [0,0,0]); "
                   "a correctness rehearsal of the C-side split, the helpers share the proving GPU"}
    try:
        for k in (1, 2):
            hip.init_devices([0] * (1 + k))
            pr.attach_helpers(k)
            pr.rounds_dev(polys, chal, rnd)
            t = []
            for _ in range(reps):
                t0 = time.perf_counter()
                o = pr.rounds_dev(polys, chal, rnd)
                t.append(time.perf_counter() - t0)
            t.sort()
            out["devices_%d" % (1 + k)] = {"median_ms": round(t[len(t) // 2] * 1e3, 3),
                                           "matches_oracle": _prove_golden(n, o)}
            pr.attach_helpers(0)
    finally:
        hip.init_devices([0])
        pr.close()
    return out


def prove_split_component(torch, hip, dev, dist, rank, world, gloo, log2n=20, reps=5):
    """C5 strong-scaled over the ranks (round 3's independent poly_mul jobs spread
    across GPUs as whole jobs).  Every rank holds the same proof inputs (gen.prove_instance, seed
    51).  Rank 1 computes round 3's t_2 chain (A2 B2)(C2 z) and rank 2 the t_3 chain
    (A3 B3)(C3 z(omega x)) (src/plonk.h:432-434, 471-473) -- at N = 2 rank 1 only t_3 --
    with plk_prover_chains_dev and sends the product bytes to rank 0 (RCCL send / receive, 4 MiB
    per chain at 2^20 gates); rank 0 runs everything else and reads them after the receive
    (plk_prover_rounds_ext_dev).  Ranks >= 3 idle.  Timed: rank 0's wall time per proof, every
    proof started on all ranks by one barrier; rank 0's single-GPU proof of the same instance is
    timed beside it.  gloo (the one-GPU rehearsal): the bytes travel through host memory."""
    n = 1 << log2n
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gen
    hpolys, chal, rnd, zh, pts = gen.prove_instance(n, 51, 2 * n + 8)
    polys = [torch.from_numpy(p).to(dev) for p in hpolys]
    pr = hip.Prover(n, zh, pts)
    from plonkhip.dist import split_proof_step
    T2, T3 = hip.PLK_CHAIN_T2, hip.PLK_CHAIN_T3
    bufs = {c: torch.zeros(pr.chain_bytes(c), dtype=torch.uint8, device=dev) for c in (T2, T3)}
    st = torch.cuda.current_stream()

    def once():
        # (N = 2: rank 1 computes t_3 only, rank 0 keeps t_2 and its (a b) q_m sum group -- the
        # one-GPU pieces, prove_split_pieces, put rank 0 with t_3 received at ~0.33 ms, while one
        # helper with both chains would deliver 8 MiB after ~0.24 ms of chains)
        return split_proof_step(pr, polys, chal, rnd, bufs, rank, world, st, via_host=gloo)

    single = None
    if rank == 0:
        first = pr.rounds_dev(polys, chal, rnd)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            pr.rounds_dev(polys, chal, rnd)
            ts.append(time.perf_counter() - t0)
        single = min(ts)
    dist.barrier()
    out = once()                             # (the first send / receive sets up the peer channel)
    torch.cuda.synchronize()
    t, outs = [], []
    for _ in range(reps):
        dist.barrier()
        t0 = time.perf_counter()
        o = once()
        if rank == 0:
            t.append(time.perf_counter() - t0)
            outs.append(o)
    dist.barrier()
    pr.close()
    if rank != 0:
        return None
    t.sort()
    return {"gpus": min(world, 3), "ms": round(t[0] * 1e3, 3), "median_ms": round(t[len(t) // 2] * 1e3, 3),
            "single_gpu_ms": round(single * 1e3, 3), "speedup": round(single / t[0], 3),
            "matches_oracle": _prove_golden(n, out), "same_as_single_gpu": all(o == first for o in [out] + outs),
            "transport": "gloo through host memory (one-GPU rehearsal)" if gloo else "RCCL send / receive",
            "note": "one 2^20-gate proof strong-scaled: rank 1 computes round 3's t_2 chain (A2 B2)(C2 z) and rank "
                    "2 the t_3 chain (A3 B3)(C3 z(omega x)) (N = 2: rank 1 t_3 only) from the same inputs, "
                    "plk_prover_chains_dev, and sends the 4 MiB products to rank 0, which runs the rest "
                    "(plk_prover_rounds_ext_dev); ms = rank 0's wall time per proof, all ranks released by one "
                    "barrier; single_gpu_ms = rank 0 alone on the same instance"}


def rank_launch_cmd(argv, n, port):
    """the child command that runs this bench as n ranks on this node (torch.distributed.run, one
    process per GPU, rendezvous on 127.0.0.1): the same arguments, so every rank parses the same
    --gpus n and finds WORLD_SIZE = n"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def world_from_args(args, env):
    """(world, launch): the rank count this process belongs to, and whether it must first start
    the ranks itself.  Decided before anything imports torch or touches a GPU: a launcher's
    WORLD_SIZE that disagrees with --gpus is an error (the line would claim the wrong n_gpus)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks" % (args.gpus, world))
        return world, False
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1 (got %d)" % n)
    return n, n > 1


def launch_ranks(n):
    """start n ranks of this bench as a CHILD process (no exec: nothing here has touched the GPU,
    and the child initialises it itself); rank 0's JSON line reaches our stdout through the
    inherited stream; returns the child's exit status"""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(rank_launch_cmd(sys.argv[1:], n, port), env=env).returncode


def main():
    args = parse()
    world, spawn = world_from_args(args, os.environ)
    if spawn:
        sys.exit(launch_ranks(world))
    import torch
    import torch.distributed as dist

    import plonkhip as hip

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; PLK_DIST_BACKEND=gloo (and more ranks than GPUs) only to rehearse
    # the multi-rank path on a one-GPU box -- the driver's runs use RCCL ("nccl")
    backend = os.environ.get("PLK_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()         # (counting devices does not initialise the GPU)
    if backend == "nccl" and world > max(1, ndev):
        raise SystemExit("bench.py: %d ranks over RCCL need %d GPUs, %d visible (PLK_DIST_BACKEND=gloo rehearses "
                         "more ranks than GPUs)" % (world, world, ndev))
    gpu = local % max(1, ndev)
    torch.cuda.set_device(gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", gpu)
    tuned = hip.tune_from_env()              # PLK_TUNE (A/B runs only; empty by default)
    hip.init(gpu)
    st = torch.cuda.current_stream()

    from plonkhip.dist import finish_sharded, g1_bytes, gpu_ops, shard_range

    n = 1 << args.log2n                      # points per MSM
    strong = world > 1 and not args.weak
    lo, hi = shard_range(n, rank, world) if strong else (0, n)
    m = hi - lo                              # points this rank reads per MSM
    B = max(1, args.msm_batch)
    sets = max(2 * B, -(-args.rotate_mib * (1 << 20) // (MSM_BYTES_PER_POINT * m)))
    sets = -(-sets // B) * B                 # whole launches never wrap the rotation
    # strong: every rank builds the SAME input sets and keeps its range; weak: rank r's sets are
    # its own shards of N * 2^log2n-point MSMs
    seed_of = (lambda s: 1234 + s) if strong or world == 1 else (lambda s, r=rank: 1234 + 100003 * r + s)
    pts, sc = make_shard_sets(torch, n, lo, hi, sets, dev, seed_of)
    ops = gpu_ops(hip, st)
    K, W = args.steps, args.warmup          # steps of B MSMs (one batched launch each)
    res = torch.zeros(((W + K) * B, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)

    def launch(first, count):
        """MSMs first .. first+count-1 (result record i = res[i]), B per launch; MSM i reads
        input set i mod sets."""
        i = first
        while i < first + count:
            b = min(B, first + count - i, sets - i % sets)
            s0 = i % sets
            ops.launch(pts[s0], 3 * m, sc[s0], m, m, b, res[i:])
            i += b

    def shard_of(j):                         # MSM W*B + j of the timed region
        s0 = (W * B + j) % sets
        return pts[s0], sc[s0]

    # the finish path once on zeroed records first: torch loads its elementwise kernels lazily
    # (tens of ms on first use), which must not land in the timed region -- and not between the
    # warmup steps and the timed ones either (an idle device drops its clocks: the first timed
    # region ran ~0.13 ms slower, tools/timing_probe.py)
    finish_sharded(ops.records_to_partials(res[:B]), n, ops, lambda j: (pts[j % sets], sc[j % sets]))
    torch.cuda.synchronize()
    launch(0, max(W, 1) * B)                 # (records are re-armed by every launch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launch(W * B, K * B)
    partials = ops.records_to_partials(res[W * B:])
    g1t, folded = finish_sharded(partials, n, ops, shard_of)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if args.profile_only:
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- correctness of the timed results (outside the timed region)
    g1s = g1_bytes(g1t[:1])
    check = {}
    first_set = W * B % sets
    if rank == 0:
        # the first timed MSM recomputed on this GPU alone from its full input (every shard)
        if world == 1 or strong:
            fp, fs = make_msm_set(torch, n, dev, seed_of(first_set))
            full_logs = [one_msm_log(torch, hip, fp, fs, n, dev, st)]
        else:
            full_logs = []
            for r in range(world):
                fp, fs = make_msm_set(torch, n, dev, 1234 + 100003 * r + first_set)
                full_logs.append(one_msm_log(torch, hip, fp, fs, n, dev, st))
        want = g1_bytes(ops.exp(torch.tensor([sum(full_logs) % 102], dtype=torch.int32, device=dev)))[0]
        check["first_msm_single_gpu_recompute"] = want == g1s[0]
    if (strong or world == 1) and args.log2n == 22:
        # the reference's own answer for a 2^22-point input through the timed kernel and the same
        # finish (sharded at N > 1: every rank its point range)
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        import gen
        with open(os.path.join(ROOT, "tests", "golden", "msm.json")) as f:
            gold = json.load(f)["large"][7]
        gp, gs = gen.msm_inputs(gold["seed"], gold["n"], gold["kind"])
        sp = torch.from_numpy(gp[lo:hi].reshape(-1).copy()).to(dev)
        ss = torch.from_numpy(gs[lo:hi].copy()).to(dev)
        rec = torch.zeros((1, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
        ops.launch(sp, 0, ss, 0, hi - lo, 1, rec)
        got, _ = finish_sharded(ops.records_to_partials(rec), n, ops, lambda j: (sp, ss))
        check["golden_2^22_reference"] = g1_bytes(got)[0].hex() == gold["out"]
    irregular = int(partials[:, 1].sum().item())

    # Kernel-level timing for the roofline, on the stream the kernel runs on: one event pair
    # around L back-to-back launches of B MSMs (a pair around every launch would add its
    # own ~6 us per pair); the average includes the launch gaps, so it is an upper bound on
    # the kernel duration that rocprofv3 reports for the same command.
    L = max(8, min(64, K))
    res2 = torch.zeros((B, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    base = (W + K) * B

    def one(j):
        s0 = (base + j * B) % sets
        s0 -= s0 % B
        ops.launch(pts[s0], 3 * m, sc[s0], m, m, B, res2)

    one(0)                       # device busy before the start event (see event_avg_ms)
    e0.record(st)
    for j in range(1, L + 1):
        one(j)
    e1.record(st)
    torch.cuda.synchronize()
    avg_ms = e0.elapsed_time(e1) / L
    alg = MSM_BYTES_PER_POINT * m * B
    achieved = alg / (avg_ms * 1e-3) / 1e9
    traffic, kname = pmc_traffic(args.log2n, B, m)

    total_points = (n if strong or world == 1 else world * n) * B * K
    value = total_points / elapsed / 1e6
    line = {
        "metric": "G1-MSM Mpoint/s + NTT Gelem/s; end-to-end prove ms at 2^20 gates",
        "value": round(value, 1),
        "unit": "Mpoint/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",   # (N = 1: the mode the N > 1 runs use)
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: SRS points kG (k uniform 1..16), HF scalars uniform 0..16, %d distinct "
                "input sets (%d MiB per GPU) rotated so every step reads cold data, resident in HBM"
                % (sets, sets * MSM_BYTES_PER_POINT * m >> 20),
        "config": {"workload": "%d x 2^%d-point G1 MSMs (srs_eval_at_s) per step, one batched launch per GPU over %d "
                               "distinct input sets; %s; ONE RCCL all-reduce of the partial logs of all K steps "
                               "(plonkhip.dist.finish_sharded)" % (
                                   B, args.log2n, B,
                                   "each MSM point-range sharded over %d GPU(s) (%d points per GPU)" % (world, m)
                                   if strong or world == 1 else
                                   "every GPU owns a 2^%d-point shard of %d-GPU MSMs" % (args.log2n, world)),
                   "points_per_msm": n if strong or world == 1 else world * n, "points_per_gpu": m,
                   "msms_per_step": B, "msms_per_launch": B, "parallelism": "dp%d" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": kname,
                     "launch_ms_avg": round(avg_ms, 5), "alg_bytes_per_launch": alg,
                     "timing": "hipEvent pair around %d back-to-back launches on the kernel's "
                               "stream, opened after one primer launch is queued" % L},
        "checks": check,
        **({"tuning": tuned} if tuned else {}),
        "irregular_inputs": irregular,
        "serial_fold_fallbacks": folded,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        torch.cuda.synchronize()
        line["cpu_baseline"] = cpu_baseline(pts[first_set].cpu().numpy(), sc[first_set].cpu().numpy(),
                                            args.cpu_seconds, g1s[0])
        check["cpu_baseline_reference"] = "error" not in line["cpu_baseline"]
    comps = wanted_components(args)
    comp = {}
    if world > 1 and "prove" in comps:
        # C5 at N GPUs: replicas only (a proof's NTT work stays on one GPU).  Every rank
        # builds its prover first, then ALL ranks start their timed proofs after one barrier, so
        # the N proofs run at the same time (rank 0's other components run after this leg); each
        # rank's proof bytes are checked against the recorded answer and the check is reduced
        pc = prove_component(torch, hip, dev, 20, reps=3, barrier=dist.barrier)
        t = torch.tensor([pc["ms"], pc["median_ms"], 1.0 if pc["matches_oracle"] else 0.0,
                          1.0 if pc["deterministic"] else 0.0], dtype=torch.float64, device=dev)
        tmax, tmin = t.clone(), t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        if rank == 0:
            ms = float(tmax[0].item())
            comp["prove_2^20_gates_replicas"] = {
                "gpus": world, "ms_slowest_rank": round(ms, 3), "median_ms_slowest_rank": round(float(tmax[1].item()), 3),
                "proofs_per_s": round(world / (ms * 1e-3), 1),
                "matches_oracle_all_ranks": bool(tmin[2].item() == 1.0),
                "deterministic_all_ranks": bool(tmin[3].item() == 1.0),
                "note": "one independent 2^20-gate proof per GPU, all ranks released by one barrier and timing "
                        "concurrently, no exchange; ms = the slowest rank's best call; matches_oracle: every rank's "
                        "34 bytes equal the recorded answer of the CPU restatement (tests/golden/prove_2_20.json)"}
        # C5 strong-scaled: one proof over up to 3 GPUs (round 3's two product chains on ranks 1, 2)
        sp = prove_split_component(torch, hip, dev, dist, rank, world, backend != "nccl")
        if rank == 0:
            comp["prove_2^20_gates_split"] = sp
    if rank == 0 and comps:
        comp.update(components(torch, hip, dev, st, comps - ({"prove"} if world > 1 else set())))
        if "msm" in comps:
            lab = pts_label(m)
            comp["msm_%s_one_per_launch" % lab] = single_msm_component(torch, hip, pts, sc, m, sets, dev)
            B8 = 8
            r8 = torch.zeros((B8, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
            avg8, med8 = event_avg_ms(torch, st, lambda i: hip.msm_g1_batch_dev(
                pts[(i * B8) % sets], 3 * m, sc[(i * B8) % sets], m, m, B8, r8[0], st), 16)
            comp["msm_%s_8_per_launch" % lab] = {
                "device_us_per_launch": round(avg8 * 1e3, 2),
                "GB_s": round(MSM_BYTES_PER_POINT * m * B8 / (avg8 * 1e-3) / 1e9, 1),
                "points_per_msm": m,
                "note": "8 MSMs per launch (the prover's commitments are 9 per launch)"}
        if world == 1 and "cpu" in comps and not args.no_cpu_baseline:
            comp["cpu_reference_other"] = cpu_other_baselines(hip)
        if "msm" in comps and torch.cuda.device_count() > 1:
            # the C-side split proof over DISTINCT GPUs (tools/devices_probe.py) is unverified until it
            # has matched the recorded answer on a multi-GPU node: a missing or failed probe is a failed check
            sp = ((comp.get("host_call_msm_2^22_devices") or {}).get("all_devices") or {}).get("prove_2^20_split_from_c")
            legs = [v for k, v in (sp or {}).items() if k.startswith("gpus_")]
            check["distinct_device_split_from_c_matches_golden"] = bool(legs) and all(
                v.get("matches_golden") is True for v in legs)
    if rank == 0 and comp:
        line["components"] = comp
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
