"""The reference's OWN test programs (src/*-test.c, unmodified) built against the drop-in
headers (`make -C oracle dropin-tests`: gcc -include include/prelude.h, linked to libplonkhip).

* gf / hf / g1 / g2 / gt / pairing / constraints exercise only host code -- our restated
  include/ headers plus the reference's own gt.h / pairing.h / constraints.h -- and must pass on
  the CPU;
* poly / srs / matrix / plonk send poly_mul, srs_eval_at_s, poly_divide, poly_eval, matrix_mul and
  matrix_inv to libplonkhip: on the GPU they must pass (the reference's own assertions against
  our kernels), and without a device they must fail loudly (no CPU fallback).

The binaries are built in the container that holds /root/reference (build()); they travel to the
GPU box with the tree (oracle/_ref is git-ignored, not gpurun-ignored).  Missing binaries fail
the tests (no skip)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "dropin_tests")
HOST_ONLY = ["gf", "hf", "g1", "g2", "gt", "pairing", "constraints"]
GPU_PATH = ["poly", "srs", "matrix", "plonk"]


def run(name, env_extra=None):
    path = os.path.join(BIN, name + "-test")
    assert os.path.exists(path), "%s missing: build with `make -C oracle ref` where /root/reference exists" % path
    env = dict(os.environ)
    env.update(env_extra or {})
    return subprocess.run([path], capture_output=True, text=True, timeout=120, env=env)


@pytest.mark.parametrize("name", HOST_ONLY)
def test_reference_host_tests_pass(name):
    r = run(name)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("name", GPU_PATH)
def test_reference_gpu_tests_fail_loudly_without_a_device(name):
    r = run(name, {"HIP_VISIBLE_DEVICES": "-1", "ROCR_VISIBLE_DEVICES": "-1"})
    assert r.returncode != 0
    assert "no CPU fallback" in r.stderr or "failed on the GPU" in r.stderr, r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_PATH + HOST_ONLY)
def test_reference_suite_on_gpu(name):
    r = run(name)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
