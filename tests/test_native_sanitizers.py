"""Host C++ runtime under AddressSanitizer + UndefinedBehaviorSanitizer.

GPU sanitizers are not available on the pool; the host code is where races and overflows
would hide (process-shared barrier, ragged multi-round pieces), so it is compiled with
``-fsanitize=address,undefined`` and driven by a forked multi-process test
(csrc/host/test_host_ops.cpp).  Also builds it with ThreadSanitizer-compatible flags for the
in-process thread fan-out.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(name, flags):
    out = os.path.join(ROOT, "build", name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    srcs = [os.path.join(ROOT, "csrc", "host", f) for f in ("host_ops.cpp", "test_host_ops.cpp")]
    if os.path.exists(out) and all(os.path.getmtime(out) > os.path.getmtime(s) for s in srcs):
        return out
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-I", os.path.join(ROOT, "csrc", "include")] + flags + \
          [os.path.join(ROOT, "csrc", "host", "host_ops.cpp"), os.path.join(ROOT, "csrc", "host", "test_host_ops.cpp"),
           "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        # skip only when the toolchain cannot build ANY sanitized program; a compile error in
        # the sources is a failure
        probe = subprocess.run(["g++", "-x", "c++", "-", "-o", os.devnull] + flags, input="int main(){}",
                               capture_output=True, text=True)
        if probe.returncode != 0:
            pytest.skip("sanitizer toolchain unavailable: " + probe.stderr[-500:])
        pytest.fail("host runtime does not build with " + " ".join(flags) + ":\n" + r.stderr[-3000:])
    return out


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("p,n", [(2, 50_001), (4, 100_003), (7, 33_333)])
def test_host_runtime_asan_ubsan(p, n):
    exe = _build("test_host_ops_asan", ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(p), str(n)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "OK" in r.stdout
