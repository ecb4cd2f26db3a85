"""The -DMP4X_DEBUG build (device-side bounds asserts, tools/build_native.py --debug) runs the
kernel paths cleanly: every MP4X_DASSERT holds on real inputs."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "mp4x", "_native", "libmp4x_hip_debug.so")

SCRIPT = r'''
import torch
import mp4x.ops.native as native
from mp4x.ops import device_ops as K
from mp4x.operators import OpCode
assert native.HIP_LIB.endswith("libmp4x_hip_debug.so"), native.HIP_LIB
dev = "cuda:0"
xs = [torch.randn(100_003, device=dev) for _ in range(3)]
out = torch.empty_like(xs[0])
K.reduce_(out, xs, int(OpCode.SUM))
assert torch.allclose(out, xs[0] + xs[1] + xs[2], atol=1e-5)
keys = torch.randint(-(1 << 62), 1 << 62, (70_001,), device=dev)
vals = torch.randn(70_001, 16, device=dev)
sk, sv, counts, perm = K.partition_pack(keys, vals, 7, want_perm=True)
assert int(counts.sum()) == 70_001
k2 = torch.randint(0, 500, (20_000,), device=dev)
uk, uv, cnt = K.reduce_by_key(k2, torch.randn(20_000, 8, device=dev), int(OpCode.SUM))
x = torch.randn(300_000, device=dev) * (torch.rand(300_000, device=dev) < 0.1)
m, c, v, nnz, bs = K.zs_encode(x, [(0, 100_000), (100_000, 200_000)])
o = torch.empty_like(x)
K.zs_decode(m, c, v, [(0, 100_000), (100_000, 200_000)], o)
assert torch.equal(o, x)
q, s = K.quant_fp8(xs[0][:100_000])
torch.cuda.synchronize()
print("debug-build-ok")
'''


def test_debug_build_kernels_hold_their_asserts():
    if not os.path.exists(DEBUG_LIB):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build_native.py"), "--debug"], cwd=ROOT,
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stdout + r.stderr
    env = dict(os.environ, MP4X_NATIVE_DEBUG="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "debug-build-ok" in out, out[-3000:]
    assert "device assert failed" not in out
