"""The C-ABI's host code under AddressSanitizer (sanitizer build
variant; no GPU needed).

`make -C ceo-recommender_amd/csrc asan` compiles tt_abi.hip (layout, plan,
workspace and argument checks of every entry point) with
-Xarch_host -fsanitize=address together with tests/native/abi_host_check.cpp,
a driver that calls every host-decided path: parameter layouts of five
geometries, workspace sizes and step plans over nine batch sizes, the
argument errors (null pointers, B < 2 in train mode, short workspace,
unsupported shapes) and the contrastive / exchange sizes.  ASan reports any
out-of-bounds access or use-after-free on the host side.
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "ceo-recommender_amd", "csrc")
EXE = os.path.join(ROOT, "ceo-recommender_amd", "lib", "abi_host_check_asan")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_abi_host_code_under_asan():
    subprocess.run(["make", "-C", CSRC, "asan"], check=True, capture_output=True, timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_host_check: ALL OK" in r.stdout
    assert "AddressSanitizer" not in r.stderr, r.stderr
