"""Host-side sanitizer runs of the C++ runtime, each compiled here and executed
on randomized inputs:

* the text core (Levenshtein / BLEU counts) under -fsanitize=address,undefined;
* the CPU twins' pointer-level cores (csrc/include/tea_cpu_core.h: classification counts,
  binned histograms, AUROC / AUPRC rows, binary P / R counts, MSE / R2 sums) and the K5b host
  twin (csrc/runtime/rowsums_host.cpp) under -fsanitize=address,undefined, against naive
  formulas;
* the direct-RCCL watchdog bookkeeping (csrc/include/tea_watchdog.h) on a fake event source
  under -fsanitize=thread, with concurrent enqueue / wait / destroy / abort threads.

GPU AddressSanitizer is not available on this pool, so device kernels are covered by the GPU
numerics suite instead."""

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


def _run(cmd, exe, env_extra, marker):
    build = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if build.returncode != 0 and "cannot find" in build.stderr and ("asan" in build.stderr or "tsan" in build.stderr):
        pytest.skip("sanitizer runtime not installed")
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, **env_extra)
    run = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert run.returncode == 0, run.stdout[-3000:] + run.stderr[-4000:]
    assert marker in run.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_cpu_twin_cores_under_asan_ubsan() -> None:
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "cpu_core_sanitize")
        cmd = [
            "g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
            "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__",
            "-I", os.path.join(REPO, "csrc", "include"), "-I", "/opt/rocm/include",
            os.path.join(REPO, "csrc", "tests", "cpu_core_sanitize.cpp"),
            os.path.join(REPO, "csrc", "runtime", "rowsums_host.cpp"), "-o", exe,
        ]
        _run(cmd, exe, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1:verify_asan_link_order=0"},
             "cpu_core_sanitize: ok")


_CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(_CLANG), reason="ROCm clang not available")
def test_rccl_watchdog_under_tsan() -> None:
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "watchdog_tsan")
        cmd = [
            _CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
            "-I", os.path.join(REPO, "csrc", "include"),
            os.path.join(REPO, "csrc", "tests", "watchdog_tsan.cpp"), "-o", exe,
        ]
        _run(cmd, exe, {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}, "watchdog_tsan: ok")
