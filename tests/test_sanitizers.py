"""Host-side sanitizer run of the C++ text runtime core: compiled with
-fsanitize=address,undefined and executed on randomized inputs.  GPU AddressSanitizer is not
available on this pool, so device kernels are covered by the GPU numerics suite instead."""

import os
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_text_core_under_asan_ubsan() -> None:
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "text_core_sanitize")
        cmd = [
            "g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
            "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
            "-I", os.path.join(REPO, "csrc", "include"),
            os.path.join(REPO, "csrc", "tests", "text_core_sanitize.cpp"), "-o", exe,
        ]
        build = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if build.returncode != 0 and "cannot find" in build.stderr and "asan" in build.stderr:
            pytest.skip("libasan not installed")
        assert build.returncode == 0, build.stderr[-3000:]
        # verify_asan_link_order=0: the environment may preload other libraries
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
        run = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
        assert run.returncode == 0, run.stdout[-2000:] + run.stderr[-3000:]
        assert "text_core_sanitize: ok" in run.stdout
