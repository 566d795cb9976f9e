"""Host sanitizer build: the drop-in headers' host code and the oracle under
-fsanitize=address,undefined (oracle/sanitize_main.c, `make -C oracle sanitize`): every raw
byte value of the field ops, random / raw group elements, ragged polynomials incl. length 0,
matrices up to 17 x 17.  Any ASan / UBSan report fails the run."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_host_code_under_asan_ubsan():
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True,
                       text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sanitize ok" in r.stdout
