"""rocprofv3 driver: K6b encode at densities 0, 0.05, 1.0 (WRITE_SIZE attribution)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mp4x.ops import device_ops as K  # noqa: E402

n = 64 << 20
for d in (0.0, 0.05, 1.0):
    x = torch.randn(n, device="cuda:0") * (torch.rand(n, device="cuda:0") < d) if d < 1 else torch.randn(n, device="cuda:0")
    torch.cuda.synchronize()
    K.zs_encode(x)
    torch.cuda.synchronize()
print("ok")
