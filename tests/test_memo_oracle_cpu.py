"""The latency memo's coherence oracle (VERDICT r5 Next #3): over random interleavings of every
input of the decision — registrations, MP4X_DEVICE_ALGO, autotune pins, a new IPC instance
(the large-message one, whose error word joins every entry's fail-stop check), the graph-mode
switch (device epochs: no hit may follow), a fail-stop error word — and
calls of every memoised kind (allreduceArray, reduceArray, broadcast / gather / scatter /
all-gather copy plans, the fused reduce-scatter) with varying [from, to), dtype, operator and
scale, every fast-path HIT must launch exactly what the full path would launch at that moment:
the same schedule, instance, buffers and offsets, slot, grid and scale.

CPU, no GPU: the real ProcessCommSlave API and DeviceEngine over fake IPC instances whose native
launches are recorded (a fake launcher and library); device tensors are CPU tensors of a subclass
that reports ``is_cuda``.  The fake fast launchers are the oracle: on a hit they decode the
memoised entry the way the native fast path does (csrc/runtime/ipc_ar.hip: slot choice from the
instance state, src = out = the caller's tensor + offset, ...), then re-run the same public call
with the memo switched off and compare the full path's one recorded launch with it.

Reference: every call re-validates its ranges (ProcessCommSlave.java:1733-1763,
CommUtils.isFromToLegal :1738): a cached decision must never differ from a fresh one."""
import ctypes
import random

import pytest

torch = pytest.importorskip("torch")
hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from mp4x import Operands, Operators  # noqa: E402
from mp4x.exceptions import Mp4jException  # noqa: E402
from mp4x.ops import native  # noqa: E402
from mp4x.parallel import ipc as ipc_mod  # noqa: E402
from mp4x.parallel import ipc_forms as forms_mod  # noqa: E402

P = 4


class Tensor(torch.Tensor):
    """A CPU tensor the engine takes for a device tensor (``is_cuda``); named and placed so the
    API's ``_is_device_tensor`` check accepts it."""

    @property
    def is_cuda(self):
        return True


Tensor.__module__ = "torch.fake"


def _dev(n, dtype):
    return torch.zeros(n, dtype=dtype).as_subclass(Tensor)


class _Log(list):
    pass


LOG = _Log()


class _FakeLib:
    """Every native entry the full paths call: recorded (launches; the pure ``*_check`` refusal
    checks launch nothing), success."""

    def __getattr__(self, name):
        if not name.startswith("mp4x_"):
            raise AttributeError(name)

        def f(*a):
            if not name.endswith("_check"):
                LOG.append((name, a))
            return 0
        return f


def _arr_vals(arr, n):
    return [int(x) for x in list(arr)[:n]]


class World:
    """One rank (rank 0 of P) of a job: the API object, its engine, fake IPC instances."""

    def __init__(self, monkeypatch):
        from mp4x.parallel.coll import LoopbackHub, _FakeComm
        from mp4x.parallel.device_engine import DeviceEngine
        from mp4x.parallel.process_comm import ProcessCommSlave, _FaultInjector
        self.mp = monkeypatch
        self.insts = []
        self.failures = []
        self.hits = {"allreduce": 0, "plan": 0, "rs": 0}
        self.graph_at = None
        for mod in (ipc_mod, forms_mod):
            monkeypatch.setattr(mod, "stream_ptr", lambda *a: 0)
        monkeypatch.setattr(native, "stream_ptr", lambda *a: 0)
        monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
        monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
        monkeypatch.setattr("mp4x.parallel.device_engine.capturing_now", lambda: False)
        monkeypatch.setattr("mp4x.parallel.engine_rooted.capturing_now", lambda: False)
        monkeypatch.setattr("mp4x.parallel.autotune.capturing_now", lambda: False)
        monkeypatch.setattr(ipc_mod, "capturing_now", lambda: False)
        monkeypatch.setattr(ipc_mod.torch, "full", lambda *a, **k: torch.zeros(1, dtype=torch.int32))
        from mp4x.ops import device_ops
        for name in ("scale_", "reduce_", "reduce_strided_", "segment_copy_", "gather_rows_"):
            if hasattr(device_ops, name):
                monkeypatch.setattr(device_ops, name, (lambda nm: lambda *a, **k: LOG.append((nm, a)))(name))
        world = self

        class _Lx:
            def allreduce_ex(self, *a):
                LOG.append(("allreduce_ex", a))
                return 0

            def fast_allreduce(self, ent, stream, base=None):
                return world.oracle("allreduce", ent, base)

            def fast_plan(self, ent, stream, base):
                return world.oracle("plan", ent, base)

            def fast_rs(self, ent, stream, base):
                return world.oracle("rs", ent, base)
        self.lx = _Lx()
        monkeypatch.setattr(native, "launch_ext", lambda: self.lx)
        monkeypatch.setattr(ipc_mod, "IpcAllreduce", self._make_inst_cls())
        eng = DeviceEngine(_FakeComm(0, P), coll=LoopbackHub(P).coll(0), device="cpu")
        eng.coll = self._fake_coll()
        eng.backend = "nccl"
        eng.device = torch.device("cuda", 0)
        eng.ipc_enabled = True
        eng._ipc_self_test = lambda inst: None
        eng._probe_instance = lambda inst, **k: []
        eng.barrier = lambda *a, **k: None
        self.eng = eng
        assert eng.ipc() is not None
        comm = object.__new__(ProcessCommSlave)
        comm.slaveNum, comm.rank = P, 0
        comm._device_engine = eng
        comm._fault = _FaultInjector(0)
        comm.stats = {"calls": {}, "bytes": 0}
        from mp4x.utils.trace import Tracer
        comm.tracer = Tracer(0)
        comm._fast_ar = comm._fast_pl = comm._fast_rs = None
        comm._enable_fast_path()
        assert comm._fast_ar is eng._fast_ar and comm._fast_pl is not None and comm._fast_rs is not None
        comm._fast_stream = lambda: 0
        comm._fast_tensor = Tensor
        self.comm = comm
        self.call = None

    # ---------------------------------------------------------------- fakes
    def _fake_coll(self):
        class _Coll:
            backend = "nccl"
            gather_into_tensor_ok = reduce_scatter_ok = True

            def __getattr__(self, name):
                def f(*a, **k):
                    LOG.append(("coll." + name, a))
                return f
        return _Coll()

    def _make_inst_cls(self):
        world = self
        cls = ipc_mod.IpcAllreduce

        def make(comm, nbytes=None, tag="default", slots=True):
            inst = object.__new__(cls)
            k = len(world.insts)
            inst.comm, inst.rank, inst.p, inst.tag = comm, 0, P, tag
            inst.lib = _FakeLib()
            inst.device, inst.cus, inst.spin_s = 0, 256, 600.0
            inst.nbytes = int(nbytes or (64 << 20))
            sb = ipc_mod.SLOT_BYTES if slots else 0
            inst._slot_bytes, inst._slot_base, inst._slot_vecs = sb, inst.nbytes // 16, sb // 16
            inst._vmm_data, inst._data_regions = False, []
            inst.share, inst.shared_gpu, inst.grid_caps, inst._cap_fast = 1, False, {}, {}
            base = 0x10_0000_0000 * (k + 1)
            inst.data_ptrs = [base + r * 0x1_0000_0000 for r in range(P)]
            inst.sig_ptrs = [base + 0x8000_0000 + r * 0x1_0000_0000 for r in range(P)]
            inst._data = ctypes.c_void_p(inst.data_ptrs[0])
            inst._sig = ctypes.c_void_p(inst.sig_ptrs[0])
            inst._pp_data = native.ptr_array(inst.data_ptrs)
            inst._pp_sig = native.ptr_array(inst.sig_ptrs)
            inst._pp_data_addr = ctypes.addressof(inst._pp_data[1])
            inst._pp_sig_addr = ctypes.addressof(inst._pp_sig[1])
            inst._herr_buf = (ctypes.c_uint32 * 1)(0)
            inst._herr = ctypes.c_void_p(ctypes.addressof(inst._herr_buf))
            inst._herr_word = None
            inst._epoch_box = (ctypes.c_uint32 * 1)(2)
            inst._fast_state = inst.on_change = inst._pp_hi = inst._copy_stream = None
            inst._epoch_dev = inst._sig_stream = None
            inst._overlap_default, inst._fuse_copy = False, True
            inst._regs, inst._peer_bases, inst._peer_refs = {}, {}, {}
            inst._scratch_pool, inst._scratch_size, inst._vmm_pool, inst._chunk_pool = {}, {}, {}, None
            inst._opened = []
            inst._order = type("NullOrder", (), {"addr": 0, "enter": staticmethod(lambda st: None)})()
            inst.close = lambda sync=True, collective=False: None
            inst.set_spin = lambda seconds, on_current_stream=True: None
            world.insts.append(inst)
            return inst
        return make

    # ---------------------------------------------------------------- state changes
    def register(self, t):
        inst = self.eng._ipc_obj
        key = (t.data_ptr(), t.numel() * t.element_size())
        if key in inst._regs:
            return
        reg = ipc_mod._Reg(keep=t)
        reg.peers = [t.data_ptr() + r * 0x4000_0000 for r in range(P)]
        reg.scratch = None
        inst._regs[key] = reg                      # (what IpcAllreduce.register leaves behind)
        inst._changed()

    def deregister(self, t):
        inst = self.eng._ipc_obj
        if inst._regs.pop((t.data_ptr(), t.numel() * t.element_size()), None) is not None:
            inst._changed()

    # ---------------------------------------------------------------- the oracle
    def oracle(self, kind, ent, base):
        from mp4x.parallel.ipc import FastAr
        herr_words = [i._herr.value for i in self.eng._ipc_all()]
        if any(ctypes.c_uint32.from_address(w).value for w in herr_words):
            return 1003                            # (the native prologue's fail-stop check)
        state = FastAr.from_address(ent.state)
        if kind == "allreduce":
            off = ent.offset
            nb = ent.nbytes
            slotted = ent.algo in (0, 1) and state.slot_vecs > 0 and 0 < nb and nb // 16 <= state.slot_vecs
            want = ("allreduce_ex", ent.algo, ent.dtype, ent.op, state.data_ptrs, state.signal_ptrs, state.rank,
                    state.p, nb, base + off, base + off, ent.blocks, None, ent.scale,
                    state.slot_base if slotted else 0, state.slot_vecs if slotted else 0)
        elif kind == "plan":
            stage = _arr_vals((ctypes.c_int64 * max(1, 4 * ent.nstage)).from_address(ent.stage), 4 * ent.nstage)
            pull = _arr_vals((ctypes.c_int64 * max(1, 4 * ent.npull)).from_address(ent.pull), 4 * ent.npull)
            want = ("mp4x_ipc_copy_plan", state.data_ptrs, state.signal_ptrs, state.rank, state.p, stage,
                    ent.nstage, pull, ent.npull, base + ent.src_off if ent.src_off >= 0 else None,
                    base + ent.out_off if ent.out_off >= 0 else None, ent.grid_len, ent.buf_vecs, ent.blocks)
        else:
            lo = _arr_vals((ctypes.c_int64 * P).from_address(ent.seg_lo), P)
            hi = _arr_vals((ctypes.c_int64 * P).from_address(ent.seg_hi), P)
            want = ("mp4x_ipc_reduce_scatter_from", ent.dtype, ent.op, state.data_ptrs, state.signal_ptrs,
                    state.rank, state.p, lo, hi, base + ent.src_off, base + ent.out_off, ent.blocks)
        words = sorted(w for w in state.herr if w)
        # the full path, now: the same public call with the memo switched off
        del LOG[:]
        saved = self.comm._fast_ar
        self.comm._fast_ar = None
        try:
            self.call()
        finally:
            self.comm._fast_ar = saved
        got = [x for x in LOG if not x[0].startswith("mp4x_ipc_bump")]
        self.hits[kind] += 1
        full = None
        if len(got) == 1:
            name, a = got[0]
            if name == "allreduce_ex" and len(a) == 17:
                full = (name, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[11], a[12], a[13],
                        a[15], a[16])
            elif name == "mp4x_ipc_copy_plan":
                pp = ctypes.cast(a[0], ctypes.c_void_p).value
                ps = ctypes.cast(a[1], ctypes.c_void_p).value
                full = (name, pp, ps, a[2], a[3], _arr_vals(a[4], 4 * a[5]), a[5], _arr_vals(a[6], 4 * a[7]), a[7],
                        a[8], a[9], a[10], a[11], a[13])
                if a[14] is not None:
                    full = full + ("device epoch",)
            elif name == "mp4x_ipc_reduce_scatter_from":
                pp = ctypes.cast(a[2], ctypes.c_void_p).value
                ps = ctypes.cast(a[3], ctypes.c_void_p).value
                full = (name, a[0], a[1], pp, ps, a[4], a[5], _arr_vals(a[6], P), _arr_vals(a[7], P), a[8], a[9],
                        a[11])
                if a[12] is not None:
                    full = full + ("device epoch",)
        if full is None or tuple(full) != tuple(want):
            self.failures.append({"kind": kind, "fast": want, "full": got if full is None else full})
        if sorted(herr_words) != words:
            self.failures.append({"kind": kind, "stale_error_words": (words, sorted(herr_words))})
        if any(i._epoch_dev is not None for i in self.eng._ipc_all()):
            self.failures.append({"kind": kind, "hit_in_graph_mode": True})
        return 0


TENSORS = [(1024, torch.float32), (65536, torch.float32), (1 << 20, torch.float32), (4096, torch.float64),
           (8192, torch.int32), (16384, torch.bfloat16), (3 << 20, torch.float32), (2048, torch.int64)]
OPS = {torch.float32: ("Float", ("SUM", "MAX", "PROD")), torch.float64: ("Double", ("SUM", "MIN")),
       torch.int32: ("Int", ("SUM", "BITS_XOR", "MAX")), torch.bfloat16: ("BFloat16", ("SUM", "MAX")),
       torch.int64: ("Long", ("SUM", "BITS_AND", "INT_MAX_LOC"))}
OPERANDS = {torch.float32: Operands.FLOAT_OPERAND, torch.float64: Operands.DOUBLE_OPERAND,
            torch.int32: Operands.INT_OPERAND, torch.bfloat16: Operands.BF16_OPERAND, torch.int64: Operands.LONG_OPERAND}


def _ranges(rng, n, es):
    """A [from, to) range: the whole tensor, a 16-byte aligned slice or an arbitrary one."""
    v = 16 // es
    r = rng.random()
    if r < 0.4:
        return 0, n
    if r < 0.75:
        a = rng.randrange(0, n // v) * v
        b = rng.randrange(a // v + 1, n // v + 1) * v
        return a, b
    a = rng.randrange(0, n - 1)
    return a, rng.randrange(a + 1, n + 1)


def _split(rng, frm, to, aligned_v):
    """p contiguous segments of [frm, to) (counts), on the 16-byte grid or not."""
    n = to - frm
    cuts = sorted(rng.randrange(0, n + 1) for _ in range(P - 1))
    if aligned_v and rng.random() < 0.7:
        cuts = sorted(min(n, c // aligned_v * aligned_v) for c in cuts)
    edges = [0] + cuts + [n]
    return [edges[i + 1] - edges[i] for i in range(P)]


def run_steps(world, rng, steps):
    pool = [_dev(n, dt) for n, dt in TENSORS]
    eng, comm = world.eng, world.comm
    from mp4x.parallel.autotune import _tune_key
    for step in range(steps):
        a = rng.random()
        if a < 0.05:
            world.register(pool[rng.randrange(len(pool))])
        elif a < 0.09:
            world.deregister(pool[rng.randrange(len(pool))])
        elif a < 0.12:
            eng.algo = rng.choice(["auto", "auto", "auto", "ipc1", "ipc2", "rccl", "a2a"])
        elif a < 0.16:
            n, dt = TENSORS[rng.randrange(len(TENSORS))]
            cls, ops = OPS[dt]
            op = getattr(getattr(Operators, cls), rng.choice(ops))
            from mp4x.operators import for_dtype, dtype_of_torch
            opr = for_dtype(op, dtype_of_torch(dt))
            eng._tuned[_tune_key(dt, opr, n * torch.empty((), dtype=dt).element_size())] = \
                rng.choice(["rccl", "ipc1", "ipc2", "a2a"])
        elif a < 0.17:
            eng._tuned.clear()
        elif a < 0.175 and eng._ipc_large is None:
            eng.ipc_large()                         # a new instance: its error word joins the fast path
        elif a < 0.18:
            inst = eng._ipc_obj
            inst._herr_buf[0] = 1                   # an earlier collective timed out
            try:
                comm.allreduceArray(pool[0], Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, 1024)
                world.failures.append({"fail_stop": "no raise"})
            except Mp4jException:
                pass
            assert inst._herr_buf[0] == 0
        elif step == int(steps * 0.95):
            eng._ipc_obj.prepare_graph()            # the graph-mode switch (device epochs from now on)
            world.graph_at = step
        else:
            k = rng.randrange(len(pool))
            t = pool[k]
            n, dt = TENSORS[k]
            es = t.element_size()
            cls, ops = OPS[dt]
            op = getattr(getattr(Operators, cls), rng.choice(ops))
            opnd = OPERANDS[dt]()
            kind = rng.choice(["allreduce", "allreduce", "reduce", "broadcast", "gather", "scatter", "allgather",
                               "reduce_scatter"])
            frm, to = _ranges(rng, n, es)
            scale = rng.choice([1.0, 1.0, 0.5]) if dt in (torch.float32, torch.float64, torch.bfloat16) else 1.0
            root = rng.randrange(P)
            if kind == "allreduce":
                call = lambda: comm.allreduceArray(t, opnd, op, frm, to, scale=scale)   # noqa: E731
            elif kind == "reduce":
                call = lambda: comm.reduceArray(t, opnd, op, frm, to, root)   # noqa: E731
            elif kind == "broadcast":
                call = lambda: comm.broadcastArray(t, opnd, frm, to, root)   # noqa: E731
            else:
                counts = _split(rng, frm, to, 16 // es)
                froms = [frm + sum(counts[:i]) for i in range(P)]
                tos = [froms[i] + counts[i] for i in range(P)]
                if kind == "gather":
                    call = lambda: comm.gatherArray(t, opnd, froms, tos, root)   # noqa: E731
                elif kind == "scatter":
                    call = lambda: comm.scatterArray(t, opnd, froms, tos, root)   # noqa: E731
                elif kind == "allgather":
                    call = lambda: comm.allgatherArray(t, opnd, froms, tos)   # noqa: E731
                else:
                    call = lambda: comm.reduceScatterArray(t, opnd, op, frm, counts)   # noqa: E731
            world.call = call
            call()
            # repeat the same call right away half of the time: the memo's hits
            if rng.random() < 0.5:
                call()


@pytest.mark.parametrize("seed", [0, 1])
def test_memo_oracle_random_walk(monkeypatch, seed):
    world = World(monkeypatch)
    run_steps(world, random.Random(seed), 1200)
    assert not world.failures, world.failures[:3]
    assert world.graph_at is not None and world.eng._ipc_obj._epoch_dev is not None
    assert world.hits["allreduce"] > 50 and world.hits["plan"] > 20 and world.hits["rs"] >= 3, world.hits


def test_the_oracle_catches_a_stale_memo(monkeypatch):
    """Teeth: with the memo never cleared (every invalidation a no-op) the same walk serves stale
    launches, and the oracle reports them."""
    from mp4x.parallel.device_engine import _FastMemo
    monkeypatch.setattr(_FastMemo, "clear", lambda self: None)
    world = World(monkeypatch)
    run_steps(world, random.Random(0), 1200)
    assert world.failures, world.hits


@settings(max_examples=12, deadline=None, suppress_health_check=list(HealthCheck))
@given(seed=st.integers(min_value=2, max_value=2 ** 31), steps=st.integers(min_value=150, max_value=260))
def test_memo_oracle_property(seed, steps):
    mp = pytest.MonkeyPatch()
    try:
        world = World(mp)
        run_steps(world, random.Random(seed), steps)
        assert not world.failures, world.failures[:3]
    finally:
        mp.undo()
