"""rocprofv3 --pmc driver for the LDS-staged kernels: K4b partition pack (LDS multisplit) and
K6b zero-suppression compaction / expansion (LDS-staged coalesced I/O)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mp4x.ops import device_ops as K  # noqa: E402

dev = "cuda:0"
pk = torch.randint(0, 1 << 62, (1_600_000,), device=dev, dtype=torch.int64)
pv = torch.randn(1_600_000, 64, device=dev)
n = 64 << 20
x = torch.randn(n, device=dev) * (torch.rand(n, device=dev) < 0.05)
o = torch.empty_like(x)
for _ in range(3):
    K.partition_pack(pk, pv, 8)
    m, c, v, nnz, bs = K.zs_encode(x)
    K.zs_decode(m, c, v, [(0, n)], o)
torch.cuda.synchronize()
assert torch.equal(o, x)
print("ok")
