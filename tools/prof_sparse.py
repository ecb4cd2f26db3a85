"""rocprofv3 driver: the sparse pipeline kernels (K4b pack, K5 reduce-by-key, K8 dedupe) on
BASELINE config-4 shapes (8 ranks x 200 k keys x 64 f32 at the owner = 1.6 M rows)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mp4x.ops import device_ops as K  # noqa: E402
from mp4x.operators import OpCode  # noqa: E402

dev = "cuda:0"
keys = torch.randint(0, 400_000, (1_600_000,), device=dev, dtype=torch.int64)
vals = torch.randn(1_600_000, 64, device=dev)
pk = torch.randint(0, 1 << 62, (200_000,), device=dev, dtype=torch.int64)
pv = torch.randn(200_000, 64, device=dev)
for _ in range(10):
    K.reduce_by_key(keys, vals, int(OpCode.SUM))
    K.partition_pack(pk, pv, 8)
    K.reduce_by_key(keys, vals, 11)
torch.cuda.synchronize()
print("ok")
