"""The host-buffer C ABI (what the drop-in headers call) from several threads at once: calls are
serialised by the library's mutex and share its staging buffers (one stream synchronize per call,
capi.hip Stage), so every result must equal the oracle's whatever the interleaving.  ctypes
releases the GIL around each call, so the threads really overlap."""
import threading

import pytest

import gen

pytestmark = pytest.mark.gpu


def test_concurrent_host_calls(hip, oracle):
    cases = []
    for i in range(12):
        pts, sc = gen.msm_inputs(100 + i, 1000 + 997 * i, "full")
        a, b = gen.poly_inputs(200 + i, 50 + 611 * i, 40 + 389 * i)
        cases.append((pts, sc, oracle.msm(pts, sc), a, b, oracle.poly_mul_ntt(a, b),
                      [int(oracle.poly_eval(a, 3)), int(oracle.poly_eval(b, 5))]))
    errors = []

    def worker(t):
        try:
            for rep in range(6):
                for j, (pts, sc, want_msm, a, b, want_pm, want_ev) in enumerate(cases):
                    if (j + t + rep) % 3 == 0:
                        assert hip.msm_g1(pts, sc) == want_msm, ("msm", t, j)
                    elif (j + t + rep) % 3 == 1:
                        assert hip.poly_mul(a, b) == want_pm, ("poly_mul", t, j)
                    else:
                        ys = hip.poly_eval_batch([a, b], [3, 5])
                        assert list(ys) == want_ev, ("poly_eval", t, j, list(ys), want_ev)
        except Exception as e:   # noqa: BLE001 (reported below)
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]
