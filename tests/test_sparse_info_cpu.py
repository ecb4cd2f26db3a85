"""The count exchange of the device sparse collectives carries every rank's key range
(mp4x/parallel/sparse.py _owner_info / _split_info), so the reduce-by-key's radix sort runs over
the bits the received keys need.  CPU: the rows and the width rule."""
import pytest

torch = pytest.importorskip("torch")

from mp4x.parallel import sparse  # noqa: E402


def test_owner_info_appends_the_key_range():
    keys = torch.tensor([5, 1_000_003, 7, 42], dtype=torch.int64)
    hist = torch.tensor([3, 1], dtype=torch.int64)
    assert sparse._owner_info(keys, hist).tolist() == [3, 1, 5, 1_000_003]
    assert sparse._owner_info(keys[:0], hist * 0).tolist() == [0, 0, 0, 0]      # empty rank: neutral


@pytest.mark.parametrize("rows,bits", [
    ([[3, 1, 5, 1_000_003], [0, 2, 0, 9]], 20),           # max 1,000,003 < 2**20
    ([[3, 1, 5, 255], [0, 0, 0, 0]], 8),                  # an empty rank does not widen it
    ([[1, 1, 0, 0], [1, 1, 0, 0]], 1),                    # only key 0: one bit
    ([[1, 1, -4, 9], [2, 0, 1, 3]], None),                # a negative key: the full signed width
    ([[1, 0, 0, (1 << 63) - 1]], 63),
])
def test_split_info(rows, bits):
    mat, got = sparse._split_info(rows, len(rows[0]) - 2)
    assert mat == [r[:-2] for r in rows]
    assert got == bits
