"""Probe of HIP stream semantics the split-proof stand-in relies on (one GPU):
1. does an event recorded on torch's current (null) stream wait for work on a NON-BLOCKING
   stream created by the library (hipStreamNonBlocking)?
2. does a torch side stream run concurrently with such a stream (or serialise behind it)?
Prints wall times in ms."""
import ctypes as C
import sys
import time

import torch

hip = C.CDLL("libamdhip64.so.7")
torch.cuda.init()
x = torch.zeros(1, device="cuda")
torch.cuda.synchronize()
CYC = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000


def nb_stream():
    s = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0
    return torch.cuda.ExternalStream(s.value)


def t_sleep_alone():
    t0 = time.perf_counter()
    torch.cuda._sleep(CYC)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


print("sleep(%d) alone on null: %.2f ms" % (CYC, t_sleep_alone()))
A = nb_stream()
# 1. A sleeps; an event on null right after: when does it complete?
with torch.cuda.stream(A):
    torch.cuda._sleep(CYC)
e = torch.cuda.Event()
t0 = time.perf_counter()
e.record(torch.cuda.current_stream())
e.synchronize()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("null-stream event after A's sleep: done after %.2f ms (A done after %.2f ms)" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3))
# 2. A sleeps; a side stream does a tiny op right after: done before A?
side = torch.cuda.Stream()
with torch.cuda.stream(A):
    torch.cuda._sleep(CYC)
t0 = time.perf_counter()
with torch.cuda.stream(side):
    x.add_(1)
es = torch.cuda.Event()
es.record(side)
es.synchronize()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("side-stream op after A's sleep: done after %.2f ms (A done after %.2f ms)" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3))
# 3. the stand-in's send: null sleeps; A waits for null then sleeps (the chain); side waits for
# an event on null (after null's sleep) and copies: does the copy finish before A's sleep ends?
torch.cuda._sleep(CYC)
en = torch.cuda.Event()
en.record(torch.cuda.current_stream())
A.wait_event(en)
with torch.cuda.stream(A):
    torch.cuda._sleep(CYC)
    ea = torch.cuda.Event()
    ea.record(A)
ev = torch.cuda.Event()
ev.record(torch.cuda.current_stream())
side.wait_event(ev)
t0 = time.perf_counter()
with torch.cuda.stream(side):
    x.add_(1)
es = torch.cuda.Event()
es.record(side)
es.synchronize()
t1 = time.perf_counter()
ea.synchronize()
t2 = time.perf_counter()
print("stand-in send pattern: side copy done after %.2f ms, A's chain after %.2f ms" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3))
print("done")
