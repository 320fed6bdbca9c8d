"""Host-side race / memory-error detection for the native runtime: the
csrc/tests/runtime_stress.cpp concurrency stress (sync barrier, async staleness, shm mailbox)
built with ThreadSanitizer and with AddressSanitizer+UBSan. GPU sanitizers are not used."""
import os
import shutil
import subprocess

import pytest

from .test_ps_cpu import ROOT

SRC = [os.path.join(ROOT, "csrc", "tests", "runtime_stress.cpp"), os.path.join(ROOT, "csrc", "runtime", "ps_core.cpp"),
       os.path.join(ROOT, "csrc", "runtime", "mailbox.cpp")]


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_runtime_stress_under_sanitizer(san, tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / f"stress_{san.split(',')[0]}"
    b = subprocess.run([cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", *SRC,
                        "-lrt", "-lpthread", "-o", str(exe)], capture_output=True, text=True)
    if b.returncode != 0 and "cannot find" in b.stderr:
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime stress: all ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
