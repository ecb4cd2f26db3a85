"""Tiny driver for rocprofv3: K6b encode/decode of 256 MiB f32 at 5 % density."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mp4x.ops import device_ops as K

n = 64 << 20
x = torch.randn(n, device="cuda") * (torch.rand(n, device="cuda") < 0.05)
for _ in range(10):
    m, c, v, nnz, bs = K.zs_encode(x)
    o = torch.empty_like(x)
    K.zs_decode(m, c, v, [(0, n)], o)
torch.cuda.synchronize()
assert torch.equal(o, x)
print("ok")
