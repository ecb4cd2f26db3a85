"""CPU unit tests of the IPC tier's policies (no GPU): the operator matrix it serves and the
selection that follows from it, the co-residency grid-cap arithmetic, the spin-bound defaults,
and the fail-stop checks at the call boundary."""
import os

import pytest
import torch

from mp4x import Operands, Operators
from mp4x.exceptions import Mp4jException
from mp4x.operators import OpCode
from mp4x.parallel import ipc as ipc_mod
from mp4x.parallel import occupancy as occ
from mp4x.parallel.device_engine import DeviceEngine, _TunedTable

ALL = {
    "Double": (torch.float64, ("SUM", "MAX", "MIN", "PROD", "FLOAT_MAX_LOC", "FLOAT_MIN_LOC")),
    "Float": (torch.float32, ("SUM", "MAX", "MIN", "PROD")),
    "Long": (torch.int64, ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD", "INT_MAX_LOC",
                           "INT_MIN_LOC")),
    "Int": (torch.int32, ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD")),
    "Short": (torch.int16, ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD")),
    "Byte": (torch.int8, ("SUM", "MAX", "MIN", "BITS_AND", "BITS_OR", "BITS_XOR", "PROD")),
    "BFloat16": (torch.bfloat16, ("SUM", "MAX", "MIN", "PROD")),
    "Half": (torch.float16, ("SUM", "MAX", "MIN", "PROD")),
}


def test_ipc_serves_the_whole_operator_table():
    for cls, (dt, ops) in ALL.items():
        for name in ops:
            assert ipc_mod.ipc_op_ok(dt, getattr(getattr(Operators, cls), name)), (cls, name)
    from mp4x.operators import CustomOperator, lookup, DType
    assert not ipc_mod.ipc_op_ok(torch.float32, CustomOperator(lambda a, b: a + b))
    assert not ipc_mod.ipc_op_ok(torch.float32, lookup(DType.F32, OpCode.BAND))      # no bitwise on floats
    assert not ipc_mod.ipc_op_ok(torch.int32, lookup(DType.I32, OpCode.IMAXLOC))     # *_LOC: packed words only


def _engine(backend="nccl"):
    e = object.__new__(DeviceEngine)
    e.backend, e.device, e.ipc_enabled, e._zc = backend, torch.device("cuda", 0), True, True
    e.ipc_twoshot_max, e.ipc_oneshot_max, e.algo, e.a2a_bytes, e.p = 16 << 20, 256 << 10, "auto", 0, 8
    e._tuned, e._sel_memo, e._select_tuned = _TunedTable(), {}, False
    return e


def test_select_never_returns_a2a_for_a_builtin_op_with_a_mesh():
    """SURVEY C20 on the xGMI tier: every built-in op at p <= 8 selects an IPC kernel (one kernel
    per call) at every size; a2a only without a mesh or for custom operators."""
    e = _engine()
    opnd = Operands.DOUBLE_OPERAND()
    for cls, (dt, ops) in ALL.items():
        for name in ops:
            op = getattr(getattr(Operators, cls), name)
            for nb in (4096, 1 << 20, 64 << 20, 1 << 30):
                for kind in ("allreduce", "reduce"):
                    a = e.select(kind, nb, op, dt, opnd)
                    assert a != "a2a", (cls, name, nb, kind)
                    if not e.rccl_ok(op, dt):
                        want = "ipc1" if kind == "allreduce" and nb <= e.ipc_oneshot_max else "ipc2"
                        assert a == want, (cls, name, nb, kind, a)
    e.ipc_enabled = False
    assert e.select("allreduce", 4096, Operators.Long.BITS_OR, torch.int64, opnd) == "a2a"
    e.ipc_enabled = True
    from mp4x.operators import CustomOperator
    assert e.select("allreduce", 4096, CustomOperator(lambda a, b: a), torch.float32, opnd) == "a2a"


def test_two_ranks_take_the_one_shot_up_to_the_slot_size(monkeypatch):
    """At p = 2 the one-shot moves the same bytes as the two-shot with one barrier fewer: the
    staged allreduce takes it up to the slot size (unless MP4X_IPC_ONESHOT_MAX pins the tier);
    p > 2 keeps the 256 KiB crossover; the rooted forms' latency tier is unchanged."""
    opnd = Operands.FLOAT_OPERAND()
    SUM = Operators.Float.SUM
    e = _engine()
    e.p = 2
    e._oneshot_ar_max = ipc_mod.SLOT_BYTES
    got = {nb: e.select("allreduce", nb, SUM, torch.float32, opnd) for nb in (256 << 10, 1 << 20, 4 << 20, 8 << 20)}
    assert got == {256 << 10: "ipc1", 1 << 20: "ipc1", 4 << 20: "ipc1", 8 << 20: "ipc2"}, got
    assert e.ipc_oneshot_max == 256 << 10
    e._oneshot_ar_max = 0               # a tier attribute: the select memo follows it
    assert e.select("allreduce", 1 << 20, SUM, torch.float32, opnd) == "ipc2"


def test_select_memo_key_covers_every_tier_input():
    """a2a_bytes, hier_min_bytes, the large-data mode, the layout and the device type
    all feed _select; changing any of them must not return a stale memoised decision."""
    e = _engine()
    e.ipc_enabled = False
    opnd = Operands.FLOAT_OPERAND()
    sel = lambda: e.select("allreduce", 1 << 20, Operators.Float.SUM, torch.float32, opnd)   # noqa: E731
    assert sel() == "rccl"
    e.a2a_bytes = 1 << 10
    assert sel() == "a2a"


def test_large_reduce_scatter_of_a_non_rccl_op_takes_the_ipc_pieces():
    e = _engine()
    e._dm_large = "auto"

    class _Whole:                 # a 64 MiB int64 device range (shape facts only)
        dtype, is_cuda = torch.int64, True

        def numel(self):
            return (64 << 20) // 8

        def element_size(self):
            return 8
    whole = _Whole()
    e._dm_large_ok = lambda flat: False
    assert e._large_choice("reduce_scatter", whole, Operators.Long.BITS_XOR) == "ipc"
    assert e._large_choice("reduce_scatter", whole, Operators.Long.SUM) is None       # RCCL reduces it


def test_blocks_per_cu_follows_the_cdna4_residency_rules():
    # light kernel: waves bound by the 8-wave SIMD limit -> 4 blocks of 512 threads per CU
    assert occ.blocks_per_cu({"sgpr": 40, "vgpr": 48, "agpr": 0, "lds": 4, "occ": 8}) == 4
    # 128 VGPRs -> 4 waves/SIMD -> 2 blocks;  121 rounds up to 128 as well
    assert occ.blocks_per_cu({"sgpr": 40, "vgpr": 121, "lds": 4, "occ": 4}) == 2
    # 174 VGPRs -> 176 -> 2 waves/SIMD -> 1 block
    assert occ.blocks_per_cu({"sgpr": 46, "vgpr": 174, "lds": 4, "occ": 2}) == 1
    # SGPR-bound: 106 SGPRs -> 128 per wave -> 6 waves/SIMD (the compiler says 7) -> 3 blocks
    assert occ.blocks_per_cu({"sgpr": 106, "vgpr": 42, "lds": 4, "occ": 7}) == 3
    # LDS-bound: a 40 KB tile fits 4 blocks, 60 KB fits 2
    assert occ.blocks_per_cu({"sgpr": 40, "vgpr": 32, "lds": 60 * 1024, "occ": 8}) == 2


def test_shared_grid_cap_halves_the_resident_budget():
    assert occ.shared_grid_cap(256, 4, 1) == 256              # a GPU of its own: no cap
    assert occ.shared_grid_cap(256, 4, 8) == 64               # 256 * 2 / 8 (the r1-r3 generic budget)
    assert occ.shared_grid_cap(256, 2, 8) == 32               # the fp8 two-shot at 8 ranks (config 5)
    assert occ.shared_grid_cap(256, 3, 8) == 48               # an SGPR-bound kernel: 3 blocks per CU
    assert occ.shared_grid_cap(256, 1, 8) == 16
    assert occ.shared_grid_cap(256, 4, 2) == 256
    assert occ.shared_grid_cap(4, 1, 8) == 1                  # never 0


def test_kernel_op_mirrors_the_native_dispatch():
    assert occ.kernel_op("F32", 0) == 0 and occ.kernel_op("BF16", 1) == 1 and occ.kernel_op("F16", 2) == 2
    assert occ.kernel_op("F64", 1) == -1 and occ.kernel_op("I16", 0) == -1 and occ.kernel_op("I64", 3) == -1


def test_resource_table_parses_when_built():
    path = occ._table_path()
    if not os.path.exists(path):
        pytest.skip("native library not built")
    t = occ.load_table()
    assert t, "empty resource table"
    # every family is present, and the exact instantiation of a hot and a runtime-op kernel resolve
    fams = {k for k, _ in t}
    assert {"k_ipc_oneshot", "k_ipc_twoshot", "k_ipc_twoshot_push", "k_ipc_reduce_range", "k_ipc_gather",
            "k_ipc_copy_plan", "k_ipc_fp8_twoshot"} <= fams
    assert occ.table_bpc("twoshot", 1, "F32", 0, 8) >= 1
    assert occ.table_bpc("rs", 5, "I8", 4, 8) >= 1
    assert occ.table_bpc("fp8", 1, "F32", 0, 8) >= 1


def test_parse_resource_remarks():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bn", os.path.join(os.path.dirname(__file__), "..", "tools",
                                                                      "build_native.py"))
    bn = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bn)
    text = """x.hip:2:1: remark: Function Name: _Z2kkILi2EEvPf [-Rpass-analysis=kernel-resource-usage]
x.hip:2:1: remark:     TotalSGPRs: 8 [-Rpass-analysis=kernel-resource-usage]
x.hip:2:1: remark:     VGPRs: 4 [-Rpass-analysis=kernel-resource-usage]
x.hip:2:1: remark:     AGPRs: 0 [-Rpass-analysis=kernel-resource-usage]
x.hip:2:1: remark:     Occupancy [waves/SIMD]: 8 [-Rpass-analysis=kernel-resource-usage]
x.hip:2:1: remark:     LDS Size [bytes/block]: 512 [-Rpass-analysis=kernel-resource-usage]
"""
    assert bn.parse_resource_remarks(text) == {"_Z2kkILi2EEvPf": {"sgpr": 8, "vgpr": 4, "agpr": 0, "occ": 8,
                                                                  "lds": 512}}


def test_spin_bound_defaults_to_the_fail_stop_budget(monkeypatch):
    monkeypatch.delenv("MP4X_IPC_SPIN_S", raising=False)
    monkeypatch.delenv("MP4X_WATCHDOG_TIMEOUT", raising=False)
    assert ipc_mod.spin_default() == 600.0
    monkeypatch.setenv("MP4X_WATCHDOG_TIMEOUT", "900")
    assert ipc_mod.spin_default() == 900.0
    monkeypatch.setenv("MP4X_IPC_SPIN_S", "1")
    assert ipc_mod.spin_default() == 1.0
    assert ipc_mod.probe_spin() == 10.0


class _Inst:
    def __init__(self):
        self.word = 0
        self.spins = []

    def raise_if_failed(self):
        if self.word:
            self.word = 0
            raise Mp4jException("an earlier IPC collective timed out")

    def set_spin(self, s):
        self.spins.append(s)


def test_every_device_collective_checks_the_error_words_at_entry():
    e = _engine()
    e.watchdog = None
    e._ipc_large = e._ipc_fp8_big = e._hier = None
    e._ipc_obj = _Inst()
    e.stats = {}
    e.coll = type("C", (), {"barrier": lambda self: None})()
    e.barrier()                                   # clean: passes
    e._ipc_obj.word = 2                           # a mid barrier of an earlier call timed out
    with pytest.raises(Mp4jException, match="timed out"):
        e.barrier()
    e._ipc_obj.word = 1
    with pytest.raises(Mp4jException):
        e.allreduce(torch.zeros(4), 0, 4, Operators.Float.SUM)


def test_probing_scope_uses_the_short_bound_and_restores(monkeypatch):
    monkeypatch.delenv("MP4X_IPC_SPIN_S", raising=False)
    monkeypatch.delenv("MP4X_WATCHDOG_TIMEOUT", raising=False)
    e = _engine()
    e._ipc_obj, e._ipc_large, e._ipc_fp8_big, e._hier = _Inst(), None, None, None
    with e.probing():
        with e.probing():                         # nested tuners: set once, restored once
            late = _Inst()
            e._probe_spin(late)                   # an instance created inside the scope
        assert e._ipc_obj.spins == [10.0]
    assert e._ipc_obj.spins == [10.0, 600.0] and late.spins == [10.0]


def test_probing_scope_with_an_explicit_bound_nests(monkeypatch):
    """bench.py's baseline configs run under probing(60): a kernel that cannot complete raises
    after 60 s instead of the 600 s fail-stop budget; an autotune inside keeps ITS bound and the
    outer one comes back after it."""
    monkeypatch.delenv("MP4X_IPC_SPIN_S", raising=False)
    monkeypatch.delenv("MP4X_WATCHDOG_TIMEOUT", raising=False)
    e = _engine()
    e._ipc_obj, e._ipc_large, e._ipc_fp8_big, e._hier = _Inst(), None, None, None
    with e.probing(60):
        late = _Inst()
        e._probe_spin(late)
        with e.probing():                         # a tuner inside: the explicit outer bound stays
            pass
        with e.probing(5):
            pass
    assert e._ipc_obj.spins == [60.0, 5.0, 60.0, 600.0] and late.spins == [60.0]
    assert e._probe_depth == 0 and e._probe_s is None


def test_process_barrier_and_close_surface_a_timed_out_collective():
    from mp4x import CommMaster, ProcessCommSlave
    import tempfile
    m = CommMaster(1, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    try:
        comm = ProcessCommSlave("t", "127.0.0.1", m.port, heartbeat=False)
        eng = _engine()
        eng.device = torch.device("cpu")
        eng._ipc_obj, eng._ipc_large, eng._ipc_fp8_big, eng._hier = _Inst(), None, None, None
        eng.shutdown = eng.abort = lambda: None
        comm._device_engine = eng
        comm.barrier()
        eng._ipc_obj.word = 3
        with pytest.raises(Mp4jException):
            comm.barrier()
        eng._ipc_obj.word = 3
        with pytest.raises(Mp4jException):
            comm.close(0)                         # reported, closed with code 1, then raised
        assert comm.closed
    finally:
        code = m.stop(timeout=5)
    assert code == 1


@pytest.mark.parametrize("fails,zc,enabled,zc_vmm", [
    (["rank 1: zero_copy_memalloc_1MiB: 12 wrong elements"], True, True, False),   # memAlloc only
    (["rank 0: zero_copy_twoshot_and_plans_4MiB: 5 wrong elements",
      "rank 1: zero_copy_memalloc_1MiB: 12 wrong elements"], False, True, True),   # zero-copy: staged kept
    (["rank 0: zero_copy_twoshot_and_plans_4MiB: barrier timeout 2", "rank 1: twoshot_4MiB: 3 wrong elements"],
     True, False, True),                                                            # a core family: IPC off
    (None, True, True, True)])
def test_self_test_failure_scope(monkeypatch, fails, zc, enabled, zc_vmm):
    """A failed memAlloc self-test alone drops only the VMM-built memAlloc (registered plain
    tensors stand in); a failed zero-copy self-test drops the zero-copy forms on every rank
    (registered / memAlloc tensors then run staged); any other failure disables IPC (the verdict
    is agreed, so every rank takes the same branch)."""
    import mp4x.parallel.ipc as ipcm

    class _FakeInst:
        closed = False

        def __init__(self, comm, *a, **k):
            pass

        def close(self, *a, **k):
            _FakeInst.closed = True

    monkeypatch.setattr(ipcm, "IpcAllreduce", _FakeInst)
    e = _engine()
    e.comm, e.rank = object(), 0
    e._ipc_self_test = lambda inst: fails
    got = e.ipc()
    assert e._zc is zc and e.ipc_enabled is enabled and e._zc_vmm is zc_vmm
    assert (got is not None) is enabled and _FakeInst.closed is (not enabled)


def test_latency_fast_path_memo_is_invalidated_by_every_decision_input():
    """The allreduceArray fast path replays a memoised native launch; every input of the decision
    that produced it clears the memo: a tier attribute, the pinned table, an IPC instance's
    registrations / epoch mode (its ``on_change`` callback), capture and teardown."""
    from mp4x.parallel.autotune import _TunedTable
    e = _engine()
    e._fast_ar = {}
    e._tuned = _TunedTable()
    e._tuned.on_change = e._invalidate_fast

    def fill():
        e._fast_ar[("shape",)] = ("launch",)

    fill()
    e.algo = "auto"                      # a tier attribute (even re-assigned to the same value)
    assert not e._fast_ar
    fill()
    e._tuned[("k",)] = "rccl"            # the pinned table
    assert not e._fast_ar
    fill()
    e._tuned.clear()
    assert not e._fast_ar

    import mp4x.parallel.ipc as ipcm
    inst = object.__new__(ipcm.IpcAllreduce)
    inst.on_change = e._invalidate_fast
    fill()
    inst._changed()                      # register / deregister / memAlloc / prepare_graph / close
    assert not e._fast_ar
    # the memo keys on the tensor's address only while something is registered
    from mp4x.parallel.device_engine import _FastMemo
    e._fast_ar = _FastMemo()
    e._ipc_obj = inst
    inst._regs = {}
    inst._changed()
    assert e._fast_ar.by_ptr is False
    inst._regs = {(4096, 1 << 20): object(), (1 << 30, 4096): object()}
    inst._changed()
    assert e._fast_ar.by_ptr is True
    ak = e._fast_ar.addr_key
    assert ak(4096, 16) == 4096 and ak(8192, 64) == 8192                # inside a registered tensor
    assert ak(4000, 200) == 4000                                         # overlaps one (a [from, to) inside it)
    assert ak(0, 4096) == 0 and ak(4096 + (1 << 20), 64) == 0            # adjacent, not overlapping
    assert ak((1 << 30) - 64, 128) == (1 << 30) - 64 and ak((1 << 30) + 4096, 16) == 0
    inst._regs = {}
    inst._changed()
    assert e._fast_ar.by_ptr is False
    e._stop_watchdog = lambda: None
    e._owns_pg = False
    fill()
    e.abort()                            # teardown
    assert not e._fast_ar


def test_fast_path_memo_only_from_the_public_api(monkeypatch):
    """Direct engine callers (DDP, ThreadComm internals) never pay the memo's bookkeeping: only the
    public API's full path asks for it (``memo=True``)."""
    import inspect
    from mp4x.parallel import process_comm
    from mp4x.parallel.device_engine import DeviceEngine
    assert inspect.signature(DeviceEngine.allreduce.__wrapped__).parameters["memo"].default is False
    for name in ("reduce", "broadcast", "gather", "scatter", "allgather"):
        assert inspect.signature(getattr(DeviceEngine, name).__wrapped__).parameters["memo"].default is False, name
    assert inspect.signature(DeviceEngine.reduce_scatter.__wrapped__).parameters["memo"].default is None
    src = inspect.getsource(process_comm.ProcessCommSlave.allreduceArray)
    assert "memo=" in src and "self._fast_lx(ent, self._fast_stream(), base)" in src


def test_epochs_alternate_parity_across_the_wrap():
    """The one-shot's double-buffered slots are chosen by the epoch's parity: consecutive epochs
    must always alternate parity, also where the 30-bit counter wraps (to 2, never 0 or 1 twice)."""
    from mp4x.parallel.ipc import next_epoch
    e = 0
    seq = []
    for _ in range(6):
        e = next_epoch(e)
        seq.append(e)
    assert seq == [1, 2, 3, 4, 5, 6]
    e = 0x3FFFFFFD
    seq = []
    for _ in range(5):
        e = next_epoch(e)
        seq.append(e)
    assert seq == [0x3FFFFFFE, 0x3FFFFFFF, 2, 3, 4]
    assert all((a ^ b) & 1 for a, b in zip(seq, seq[1:]))


def test_staged_calls_take_the_slots_only_when_fused_one_piece_and_small(monkeypatch):
    """The staged allreduce passes the slot region (above the staging buffer) to the launcher for
    a one-piece, fused one- or two-shot that fits a slot, and the single-buffer form (0, 0)
    otherwise (a message larger than a slot, the unfused copy-in)."""
    calls = []

    class _Lx:
        def allreduce_ex(self, *a):
            calls.append(a)
            return 0
    monkeypatch.setattr(ipc_mod.native, "launch_ext", lambda: _Lx())
    monkeypatch.setattr(ipc_mod, "stream_ptr", lambda *a: 0)
    from mp4x.parallel import ipc_forms as forms_mod
    monkeypatch.setattr(forms_mod, "stream_ptr", lambda *a: 0)
    inst = object.__new__(ipc_mod.IpcAllreduce)
    inst.raise_if_failed = lambda: None
    entered = []
    inst._order = type("O", (), {"enter": staticmethod(entered.append)})()
    inst.nbytes, inst._slot_bytes = 1 << 20, 256 << 10
    inst._slot_base, inst._slot_vecs = (1 << 20) // 16, (256 << 10) // 16
    inst.shared_gpu, inst._epoch_dev, inst._overlap_default = False, None, False
    inst.rank, inst.p, inst._pp_data_addr, inst._pp_sig_addr = 0, 2, 0x1000, 0x2000
    inst.lib = None
    cases = ((1024, ipc_mod.ONESHOT, True, True), (65536, ipc_mod.ONESHOT, True, True),
             (65540, ipc_mod.ONESHOT, True, False), (1024, ipc_mod.TWOSHOT, True, True),
             (65540, ipc_mod.TWOSHOT, True, False),
             (1024, ipc_mod.ONESHOT, False, False))
    # an unaligned input on ONE rank must not change the protocol: it is copied to an aligned
    # temporary and still takes the slots (the decision is rank-independent)
    cases += ((1024, ipc_mod.ONESHOT, True, True, 1), (1024, ipc_mod.TWOSHOT, True, True, 1))
    for n, algo, fuse, want, *shift in cases:
        inst._fuse_copy = fuse
        if not fuse:
            inst._data = type("V", (), {"value": 0})()
            inst.lib = type("L", (), {"mp4x_memcpy_async": staticmethod(lambda *a: 0)})()
        calls.clear()
        t = torch.zeros(n + 4)[shift[0]:shift[0] + n] if shift else torch.zeros(n)
        inst.allreduce(t, Operators.Float.SUM, algo=algo, out=torch.zeros(n), capturing=False)
        (a,) = calls
        assert entered and set(entered) == {0}       # the stream order joined before the launch
        assert not fuse or (a[8] is not None and a[8] % 16 == 0), a[8]    # the fused copy-in's source
        assert a[15:] == ((inst._slot_base, inst._slot_vecs) if want else (0, 0)), (n, algo, fuse, a[15:])


def test_registered_tensors_keep_zero_copy_above_the_latency_tier_at_two_ranks(monkeypatch):
    """The two-rank one-shot extension (up to the slot size) is for staged calls: a registered
    tensor above the 256 KiB latency tier still runs the zero-copy two-shot (no staging copy)."""
    e = _engine()
    e.p = 2
    e._oneshot_ar_max = ipc_mod.SLOT_BYTES
    e.device = torch.device("cpu")
    e.stats, e.watchdog, e._hier, e._fast_ar = {}, None, None, None
    reg = torch.zeros((1 << 20) // 4)

    class _Inst:
        _epoch_dev = None

        def registered(self, view):
            return [1, 2] if view.data_ptr() == reg.data_ptr() else None
    e._ipc_obj = _Inst()
    ran = []
    monkeypatch.setattr(e, "_run_allreduce", lambda algo, view, op, scale=1.0, capturing=None: ran.append(algo))
    monkeypatch.setattr(e, "_post_scale", lambda *a: None)
    monkeypatch.setattr(e, "check_failed", lambda: None, raising=False)
    SUM, F = Operators.Float.SUM, Operands.FLOAT_OPERAND()
    for t in (reg, torch.zeros((1 << 20) // 4), torch.zeros((64 << 10) // 4)):
        e.allreduce(t, 0, t.numel(), SUM, F)
    assert ran == ["ipc2z", "ipc1", "ipc1"], ran


def test_plan_memo_records_only_one_host_epoch_launch_on_the_callers_tensor(monkeypatch):
    """DeviceEngine._plan_memo memoises a copy-plan / reduce-scatter call for the API fast path only
    when it made exactly ONE host-epoch launch that reads / writes nothing but the caller's tensor
    (a temporary for an unaligned tensor, several launches or device epochs are not replayable)."""
    import ctypes
    from mp4x.parallel.device_engine import _FastMemo
    from mp4x.ops import native
    e = _engine()
    e._fast_ar = _FastMemo()
    e._probe_depth = 0
    e._ipc_large = e._ipc_fp8_big = e._hier = None

    class _Inst:
        _plan_sink = None
        _herr = ctypes.c_void_p()

        def fast_state(self, words):
            return 4242
    inst = e._ipc_obj = _Inst()
    monkeypatch.setattr(native, "launch_ext", lambda: type("L", (), {"fast_plan": 1, "fast_rs": 1})())
    monkeypatch.setattr("mp4x.parallel.device_engine.capturing_now", lambda: False)
    arr = torch.zeros(1024)
    base, end = arr.data_ptr(), arr.data_ptr() + 4096
    sa = (ctypes.c_int64 * 4)()

    def plan(*recs):
        def fn():
            for src, out, edev in recs:
                if inst._plan_sink is not None:        # (what IpcForms._plan does)
                    inst._plan_sink.append(("plan", sa, 1, sa, 0, src, out, 64, 1 << 16, 8, edev))
            return True
        return fn
    cases = [((plan((base, None, None)),), True), ((plan((None, base + 2048, None)),), True),
             ((plan((base - 4096, None, None)),), False), ((plan((base, end, None)),), False),
             ((plan((base, None, None), (None, base, None)),), False), ((plan((base, None, 99)),), False)]
    for (fn,), want in cases:
        e._fast_ar.clear()
        assert e._plan_memo(True, "broadcast", arr, (0, 1024, 1), fn) is True
        assert (len(e._fast_ar) == 1) is want, (want, dict(e._fast_ar))
        assert inst._plan_sink is None
    e._fast_ar.clear()
    assert e._plan_memo(False, "broadcast", arr, (0, 1024, 1), plan((base, None, None))) is True
    assert not e._fast_ar                                     # engine-internal callers never memoise
    e._plan_memo(True, "broadcast", arr, (0, 1024, 1), plan((base, None, None)))
    (key, ent), = e._fast_ar.items()
    assert key == ("broadcast", 0, arr.get_device(), 1024, torch.float32, 0, 1024, 1)
    assert ent.state == 4242 and ent.src_off == 0 and ent.out_off == -1
    assert (ent.stat, ent.api) == ("broadcast.ipc", "broadcastArray")
    assert isinstance(ent, tuple) and ent[0] == 4242          # (positional: what the native launcher reads)
