"""TorchColl helpers for dtypes the transports cannot move natively (moved as their bytes)."""
import torch

from mp4x.parallel.coll import _mv, _scale


def test_split_scaling_follows_the_uint8_view():
    a = torch.zeros(10, dtype=torch.int16)
    assert _mv(a).shape == (20,)
    assert _scale([4, 6], a) == [8, 12]               # 1-D: byte splits
    rows = torch.zeros(10, 3, dtype=torch.int16)
    assert _mv(rows).shape == (10, 6)                 # only the last dim widens
    assert _scale([4, 6], rows) == [4, 6]             # row splits unchanged
    f = torch.zeros(10, dtype=torch.float32)
    assert _mv(f) is f and _scale([4, 6], f) == [4, 6]
    assert _scale(None, a) is None
