"""Memory held by the IPC mesh stays bounded (p processes sharing one GPU).

The reference's collectives work on the caller's arrays and hold no library memory between calls
(ProcessCommSlave.java:1733-1763).  mp4x maps caller tensors into every peer (registerBuffer) and
builds peer-mapped tensors (memAlloc); these tests pin that a long job which registers or
allocates many DISTINCT sizes does not grow device memory — on the owner or on any peer — and
that every result stays exact, including when a peer re-registers a new allocation at a recycled
address (the case that read wrong memory in round 2 and made rounds 2-3 keep every mapping).
Device memory is read with ``torch.cuda.mem_get_info`` (device-wide: every rank's allocations
and imports on the shared GPU count).
"""
import pytest

torch = pytest.importorskip("torch")

from spawn_ranks import run_spawn  # noqa: E402

pytestmark = pytest.mark.gpu

CYCLES = 50
BOUND = 768 << 20        # device memory growth allowed over the whole loop (all ranks together)


def _pat(n, r):
    return (torch.arange(n, device="cuda", dtype=torch.int32) % 13 + r).float()


def _exp(n, p):
    i = torch.arange(n, device="cuda", dtype=torch.int32) % 13
    return (i * p + p * (p - 1) // 2).float()


def _used():
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    return total - free


def _memalloc_cycles(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    comm.device.ipc()
    samples, bad = [], 0
    for k in range(CYCLES):
        n = (8 << 20) // 4 + k * (256 << 10)            # 8 MiB + k * 1 MiB: every size distinct
        t = comm.memAlloc(n, torch.float32)
        t.copy_(_pat(n, r))
        comm.allreduceArray(t, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
        torch.cuda.synchronize()
        bad += int((t != _exp(n, p)).sum())
        comm.memFree(t)
        del t
        torch.cuda.empty_cache()                        # temporaries of the check are not memAlloc's
        comm.barrier()
        samples.append(_used())
    return bad, samples, dict(comm.device.stats)


def _register_cycles(comm):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    comm.device.ipc()
    samples, bad, regs = [], 0, 0
    for k in range(CYCLES):
        n = (8 << 20) // 4 + k * (256 << 10)
        t = torch.empty(n, device="cuda")
        regs += int(comm.registerBuffer(t))
        t.copy_(_pat(n, r))
        comm.allreduceArray(t, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
        torch.cuda.synchronize()
        bad += int((t != _exp(n, p)).sum())
        comm.deregisterBuffer(t)
        del t
        torch.cuda.empty_cache()                        # the segment really goes back to the device
        comm.barrier()
        samples.append(_used())
    return bad, samples, regs, dict(comm.device.stats)


def _recycled(comm):
    """Every rank frees its registered tensor and allocates a new one of the same size — usually
    at the recycled address — then registers it again: the peers must read the NEW memory."""
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    comm.device.ipc()
    n = (24 << 20) // 4
    out = []
    for k in range(6):
        t = torch.empty(n, device="cuda")
        addr = t.data_ptr()
        assert comm.registerBuffer(t)
        t.copy_(_pat(n, r + 5 * k))                      # new contents every round
        comm.allreduceArray(t, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, n)
        torch.cuda.synchronize()
        exp = _exp(n, p) + 5 * k * p
        out.append((addr, int((t != exp).sum())))
        comm.deregisterBuffer(t)
        del t
        torch.cuda.empty_cache()
        comm.barrier()
    return out


@pytest.mark.parametrize("p", [2, 3])
def test_memalloc_free_cycles_of_distinct_sizes_stay_bounded(p):
    out = run_spawn(p, _memalloc_cycles, timeout=300)
    for r, (bad, samples, stats) in out.items():
        assert bad == 0, (r, bad)
        assert stats.get("allreduce.ipc2z", 0) + stats.get("allreduce.ipc2w", 0) >= CYCLES, stats
        grow = max(samples) - samples[0]
        assert grow <= BOUND, (r, grow >> 20, [s >> 20 for s in samples])


@pytest.mark.parametrize("p", [2, 3])
def test_register_deregister_cycles_of_distinct_sizes_stay_bounded(p):
    out = run_spawn(p, _register_cycles, timeout=300)
    for r, (bad, samples, regs, stats) in out.items():
        assert bad == 0, (r, bad)
        assert regs == CYCLES, regs
        grow = max(samples) - samples[0]
        assert grow <= BOUND, (r, grow >> 20, [s >> 20 for s in samples])


def test_reregistration_at_a_recycled_address_is_exact():
    out = run_spawn(4, _recycled, timeout=240)
    for r, rows in out.items():
        assert all(bad == 0 for _, bad in rows), (r, rows)
    # the point of the test: some round reused an address the peers had mapped before
    assert any(len({a for a, _ in rows}) < len(rows) for rows in out.values()), out
