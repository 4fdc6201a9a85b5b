"""Host runtime under sanitizers: the C++ self-test of the control plane / codecs / JPEG decoder
is compiled plain, with AddressSanitizer + UndefinedBehaviorSanitizer, and with ThreadSanitizer
(concurrent TCP and in-process senders), then run.  Host code only (GPU sanitizers are not
available on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "dcnn_amd", "csrc", "native")


@pytest.mark.parametrize("san", ["", "address,undefined", "thread"])
def test_native_selftest(tmp_path, san):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "selftest")
    flags = ["-O1", "-g", "-std=c++17", "-pthread"]
    if san:
        flags += [f"-fsanitize={san}", "-fno-omit-frame-pointer"]
    cmd = [cxx, *flags, os.path.join(SRC, "tests", "native_selftest.cpp"), os.path.join(SRC, "comm.cpp"),
           os.path.join(SRC, "jpeg.cpp"), "-I", SRC, "-o", exe, "-lz", "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    env.pop("LD_PRELOAD", None) if san else None
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "native selftest OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
