"""memAlloc plumbing that runs without a GPU: the chunk plan and the SCM_RIGHTS fd exchange
between real rank processes (memfd files stand in for the exported dmabuf fds)."""
import os

import pytest

from harness import run_ranks
from mp4x.exceptions import Mp4jException
from mp4x.parallel.vmm import chunk_plan


def test_chunk_plan():
    g = 2 << 20
    assert chunk_plan(1, g, 512 << 20) == (g, 1)
    assert chunk_plan(g, g, 512 << 20) == (g, 1)
    assert chunk_plan(g + 1, g, 512 << 20) == (2 * g, 1)
    assert chunk_plan(512 << 20, g, 512 << 20) == (512 << 20, 1)
    # above the cap: whole chunks of the cap, enough of them
    c, n = chunk_plan((8 << 30) + 5, g, 512 << 20)
    assert c == 512 << 20 and n == 17 and c * n >= (8 << 30) + 5
    # a cap that is not a granularity multiple is rounded down to one
    c, n = chunk_plan(10 * g, g, 3 * g + 7)
    assert c == 3 * g and n == 4
    # 4 KiB device granularity: buffers of 2 MiB and up take 2 MiB multiples
    assert chunk_plan(2796224, 4096, 8 << 20) == (4 << 20, 1)
    assert chunk_plan(5000, 4096, 8 << 20) == (8192, 1)
    assert chunk_plan((40 << 20) + 64, 4096, 8 << 20) == (8 << 20, 6)
    with pytest.raises(Mp4jException):
        chunk_plan(0, g)


def _fd_fn(comm, nfds):
    from mp4x.parallel.vmm import exchange_fds
    r, p = comm.getRank(), comm.getSlaveNum()
    mine = []
    for k in range(nfds):
        fd = os.memfd_create(f"r{r}k{k}")
        os.write(fd, f"rank{r}-chunk{k}".encode())
        mine.append(fd)
    got = exchange_fds(comm.server, r, p, mine, timeout=30)
    for fd in mine:
        os.close(fd)
    seen = {}
    for j, fds in got.items():
        vals = []
        for fd in fds:
            # pread: the received fd shares its file offset with the sender's and with every
            # other receiver's copy (one open file description), so no lseek + read
            vals.append(os.pread(fd, 64, 0).decode())
            os.close(fd)
        seen[j] = vals
    return seen


@pytest.mark.parametrize("p,nfds", [(2, 3), (4, 1), (3, 0), (2, 450)])
def test_exchange_fds(p, nfds):
    res, _, _ = run_ranks(p, _fd_fn, args=(nfds,), timeout=60)
    for r, seen in res.items():
        assert sorted(seen) == [j for j in range(p) if j != r]
        for j, vals in seen.items():
            assert vals == [f"rank{j}-chunk{k}" for k in range(nfds)], (r, j, vals[:3])
