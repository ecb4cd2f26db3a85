"""The IPC collective forms beyond allreduce, and the mesh self-tests (mixin of
:class:`~mp4x.parallel.ipc.IpcAllreduce`; split out of parallel/ipc.py in round 5).

* zero-copy reduce-scatter / all-gather / gather / scatter on registered tensors (one kernel at
  any size, the peers' own tensors);
* staged reduce-scatter / all-gather over ragged ranges and the copy-plan broadcast / scatter /
  gather (up to the staging buffer), and their piecewise forms at any size;
* the collective exact self-tests of the zero-copy forms and of a memAlloc region.

Reference: the ring reduce-scatter with fused recv + reduce (ProcessCommSlave.java:1329-1373),
the ring all-gather (:694-737), the binary-tree scatter (:1103-1159) and the dynamic-tree gather
(:440-520) — here as direct full-mesh kernels over xGMI (csrc/runtime/ipc*.hip).
"""
from __future__ import annotations

import ctypes
import logging

import torch

from ..exceptions import Mp4jException
from ..operators import dtype_of_torch
from ..ops import native
from ..ops.native import check, ptr_array, stream_ptr, c_int64, c_void_p

LOG = logging.getLogger("mp4x.ipc")

ZC_TAG = 0x80000000      # epoch tag of the zero-copy protocol (csrc/runtime/ipc.hip kZcTag)
PUSH_TAG = 0x40000000    # ... and of its push form (kPushTag); host epochs use the low 30 bits


class IpcForms:
    """Collective forms and self-tests; state (buffers, peers, epochs) lives on IpcAllreduce."""

    def selftest_zero_copy(self, n: int) -> int:
        """Collective exact-pattern run of the zero-copy two-shot, pull AND push forms (f32 SUM,
        ``n`` elements), then of the zero-copy copy plans (gather / scatter), on a dedicated plain
        device allocation per rank, mapped into every peer like a registered tensor (+ a push
        scratch); every form twice on the same memory.  Returns the number of wrong elements on
        this rank over all runs (-1: setup failed here)."""
        nbytes = n * 4
        ptr, scr, opened, err = c_void_p(), c_void_p(), [], None
        hs = self.lib.mp4x_ipc_handle_size()
        chunk = -(-(nbytes // 16) // self.p)
        try:
            check(self.lib.mp4x_dev_alloc(nbytes, ctypes.byref(ptr)), "dev_alloc")
            check(self.lib.mp4x_ipc_alloc((self.p - 1) * chunk * 16, ctypes.byref(scr)), "ipc_alloc(scratch)")
            h = ctypes.create_string_buffer(hs)
            hsc = ctypes.create_string_buffer(hs)
            check(self.lib.mp4x_ipc_get_handle(ptr, h), "ipc_get_handle(selftest)")
            check(self.lib.mp4x_ipc_get_handle(scr, hsc), "ipc_get_handle(selftest scratch)")
            blob = (h.raw, hsc.raw)
        except Exception as e:   # noqa: BLE001
            err, blob = str(e), None
        allh = self.comm.server.call("allgather_obj", self.rank, (blob, err))
        bad = -1 if any(e for _, e in allh) else 0
        peers, scrs = [], []
        if bad == 0:
            try:
                for r, (b, _) in enumerate(allh):
                    if r == self.rank:
                        peers.append(ptr.value)
                        scrs.append(scr.value)
                        continue
                    for hb, lst in ((b[0], peers), (b[1], scrs)):
                        q = c_void_p()
                        check(self.lib.mp4x_ipc_open_handle(ctypes.create_string_buffer(bytes(hb), hs),
                                                            ctypes.byref(q)), "ipc_open_handle(selftest)")
                        opened.append(q)
                        lst.append(q.value)
            except Exception:   # noqa: BLE001
                bad = -1
        oks = self.comm.server.call("allgather_obj", self.rank, bad)
        if all(o == 0 for o in oks):
            from ..operators import Operators, for_dtype, DType
            op = for_dtype(Operators.Float.SUM, DType.F32)
            got = torch.empty(n, device="cuda")
            st = self._launch_stream()
            # each form twice on new data: the second run would read any stale cache line the
            # first one left behind on this topology
            for push, salt in ((False, 0), (True, 1)):
                i = (torch.arange(n, device="cuda", dtype=torch.int32) + salt) % 13
                mine = (i + self.rank).float()
                exp = (i * self.p + self.p * (self.p - 1) // 2).float()
                check(self.lib.mp4x_memcpy_async(ptr.value, mine.data_ptr(), nbytes, st), "selftest fill")
                torch.cuda.synchronize()
                self.comm.server.call("barrier", self.rank)     # every rank's fill is done
                # twice: the second call reduces the first call's RESULT in place (as a training
                # loop does), so a stale cache line left by the first call would show
                for rep in range(2):
                    if push:
                        self._push_ptrs(nbytes, op, peers, scrs, torch.float32)
                    else:
                        self.allreduce_registered_ptrs(ptr.value, nbytes, op, peers, torch.float32)
                    check(self.lib.mp4x_memcpy_async(got.data_ptr(), ptr.value, nbytes, st), "selftest read")
                    torch.cuda.synchronize()
                    bad += int((got != exp * (self.p ** rep)).sum())
                self.comm.server.call("barrier", self.rank)     # peers are done before the refill
            bad += self._selftest_plans(ptr.value, peers, n, got, st)
        elif bad == 0:
            bad = -1
        torch.cuda.synchronize()
        self.comm.server.call("barrier", self.rank)         # every peer is done before unmapping
        for q in opened:
            native.soft_check(self.lib.mp4x_ipc_close_handle(q), "ipc_close_handle", LOG)
        from . import ipc as _ipc            # (the knob lives there; tests patch it)
        if not _ipc.UNORDERED_RELEASE:
            self._flush_translations()
            self.comm.server.call("barrier", self.rank)     # every importer unmapped before the owners free
        if ptr:
            native.soft_check(self.lib.mp4x_ipc_free(ptr), "ipc_free", LOG)
        if scr:
            native.soft_check(self.lib.mp4x_ipc_free(scr), "ipc_free", LOG)
        return bad

    def _selftest_plans(self, ptr: int, peers, n: int, got: torch.Tensor, st) -> int:
        """The zero-copy copy plans (gather / scatter pulling straight from the peers' mapped
        allocations) on the self-test allocation, each twice with fresh data written by the
        owners in between (a stale line on either side of the link shows as a wrong element).
        Returns the number of wrong elements on this rank."""
        p, r, root = self.p, self.rank, self.p - 1
        nvec = n * 4 // 16
        lo = [j * nvec // p for j in range(p)]
        ln = [(j + 1) * nvec // p - lo[j] for j in range(p)]
        bad = 0
        for salt in (2, 3):
            i = (torch.arange(n, device="cuda", dtype=torch.int32) + salt) % 13
            check(self.lib.mp4x_memcpy_async(ptr, (i + r).float().data_ptr(), n * 4, st), "selftest fill")
            torch.cuda.synchronize()
            self.comm.server.call("barrier", self.rank)
            pull = [(lo[j], lo[j], ln[j], j) for j in range(p) if j != root] if r == root else []
            self._plan_registered(peers, pull, ptr, max(ln), nvec)        # gather to root
            check(self.lib.mp4x_memcpy_async(got.data_ptr(), ptr, n * 4, st), "selftest read")
            torch.cuda.synchronize()
            exp = (i + r).float()
            if r == root:
                for j in range(p):
                    exp[lo[j] * 4:(lo[j] + ln[j]) * 4] += j - r
            bad += int((got != exp).sum())
            self.comm.server.call("barrier", self.rank)     # the gather's reads are done
            if r == root:                                   # new data at the root, then scatter
                check(self.lib.mp4x_memcpy_async(ptr, (i + 100).float().data_ptr(), n * 4, st), "selftest fill")
                torch.cuda.synchronize()
            self.comm.server.call("barrier", self.rank)
            pull = [(lo[r], lo[r], ln[r], root)] if r != root else []
            self._plan_registered(peers, pull, ptr, max(ln), nvec)        # scatter from root
            check(self.lib.mp4x_memcpy_async(got.data_ptr(), ptr, n * 4, st), "selftest read")
            torch.cuda.synchronize()
            if r != root:
                exp[lo[r] * 4:(lo[r] + ln[r]) * 4] = (i + 100).float()[lo[r] * 4:(lo[r] + ln[r]) * 4]
            else:
                exp = (i + 100).float()
            bad += int((got != exp).sum())
            self.comm.server.call("barrier", self.rank)
        return bad

    def selftest_memalloc(self, n: int) -> int:
        """Collective: memAlloc (VMM chunks exported as dmabuf fds, imported by every peer)
        tensors through the zero-copy two-shot, pull and push, each twice on the same memory (the
        second call reduces the first call's result) — in TWO alloc / free cycles of different
        sizes, so an allocation made after a memFree released memory is checked too (round 3 saw
        every later allocation's peer views read zeros after a release).  Returns this rank's wrong
        elements (-1: setup failed on some rank, agreed)."""
        from ..operators import Operators, for_dtype, DType
        op = for_dtype(Operators.Float.SUM, DType.F32)
        bad = 0
        for m in (n, n // 2 + (3 << 12)):
            try:
                t = self.mem_alloc(m * 4, torch.float32)
            except Exception:   # noqa: BLE001 — agreed inside mem_alloc (every rank raises)
                return -1
            try:
                reg, _ = self._find(t)
                for push in (False, True):
                    i = (torch.arange(m, device="cuda", dtype=torch.int32) + int(push)) % 13
                    t.copy_((i + self.rank).float())
                    exp = (i * self.p + self.p * (self.p - 1) // 2).float()
                    torch.cuda.synchronize()
                    self.comm.server.call("barrier", self.rank)
                    for rep in range(2):
                        if push and reg.scratch is not None:
                            self._push_ptrs(m * 4, op, reg.peers, reg.scratch, torch.float32)
                        else:
                            self.allreduce_registered_ptrs(t.data_ptr(), m * 4, op, reg.peers, torch.float32)
                        torch.cuda.synchronize()
                        bad += int((t != exp * (self.p ** rep)).sum())
                    self.comm.server.call("barrier", self.rank)
            finally:
                torch.cuda.synchronize()
                self.mem_free(t)
        return bad


    # ---------------------------------------------------------------- zero-copy RS / AG
    # On a registered tensor the direct reduce-scatter / all-gather kernels read the peers'
    # tensors themselves: rank r reduces segment r from every peer straight into its own
    # segment r (peers only read THEIR segment of it), or pulls every peer's segment into its
    # own tensor (peers only read ITS segment).  One launch at any size, no staging or copy-out.
    def _zc_segs(self, flat: torch.Tensor, froms, tos):
        es = flat.element_size()
        base = froms[0]
        if base < 0 or tos[-1] > flat.numel():      # (same-shaped tensors: rank-independent)
            return None
        rng = flat[base:tos[-1]]
        if not self._zc_regs_ok(rng):
            return None
        peers = self.registered(rng)
        if peers is None or rng.data_ptr() % 16:
            return None
        if not all(((f - base) * es) % 16 == 0 and ((t - base) * es) % 16 == 0 for f, t in zip(froms, tos)):
            return None
        lo = [(f - base) * es // 16 for f in froms]
        hi = [(t - base) * es // 16 for t in tos]
        return rng, peers, lo, hi

    def _zc_regs_ok(self, rng: torch.Tensor) -> bool:
        return bool(self._regs) and rng.numel() > 0 and \
            (not torch.cuda.is_current_stream_capturing() or self._epoch_dev is not None)

    def reduce_scatter_registered(self, flat: torch.Tensor, froms, tos, op) -> bool:
        z = self._zc_segs(flat, froms, tos) if self.supports(flat, op) else None
        if z is None:
            return False
        self.raise_if_failed()
        rng, peers, lo, hi = z
        r = self.rank
        st = self._launch_stream()
        edev = self._next_epoch(st)
        pp = ptr_array(peers)
        maxv = max(h - l_ for l_, h in zip(lo, hi))
        check(self.lib.mp4x_ipc_reduce_scatter(int(dtype_of_torch(flat.dtype)), int(op.code), pp[0], self._pp_sig[0],
                                               r, self.p, lo[r], hi[r], rng.data_ptr() + lo[r] * 16,
                                               self.epoch | ZC_TAG, self._grid(maxv, "rs", flat.dtype, op), edev, st),
              "mp4x_ipc_reduce_scatter(zero-copy)")
        return True

    def allgather_registered(self, flat: torch.Tensor, froms, tos) -> bool:
        z = self._zc_segs(flat, froms, tos)
        if z is None:
            return False
        self.raise_if_failed()
        rng, peers, lo, hi = z
        st = self._launch_stream()
        edev = self._next_epoch(st)
        pp = ptr_array(peers)
        lo_a = (c_int64 * self.p)(*lo)
        hi_a = (c_int64 * self.p)(*hi)
        maxv = max(h - l_ for l_, h in zip(lo, hi))
        check(self.lib.mp4x_ipc_allgather(pp[0], self._pp_sig[0], self.rank, self.p, lo_a, hi_a, rng.data_ptr(),
                                          self.epoch | ZC_TAG, self._grid(maxv, "gather"), edev, st),
              "mp4x_ipc_allgather(zero-copy)")
        return True

    # ---------------------------------------------------------------- zero-copy gather / scatter
    # The copy-plan kernel on the registered tensors themselves: pulls read the peers' tensors
    # (not their staging buffers) and land in this rank's tensor; nothing is staged.  The start
    # barrier orders the pulls after every owner's earlier writes, the end barrier keeps the
    # sources unmodified until every pull is done (as for the staged plans).  Epoch tag as the
    # other zero-copy forms: a rank running the staged plan against these fails at once.
    def _plan_registered(self, peers, pull, out_ptr, grid_len: int, buf_vecs: int) -> None:
        self.raise_if_failed()
        st = self._launch_stream()
        edev = self._next_epoch(st)
        pp = ptr_array(peers)
        sa = (c_int64 * 4)()
        pa = (c_int64 * (4 * max(1, len(pull))))(*[x for it in pull for x in it])
        check(self.lib.mp4x_ipc_copy_plan(pp[0], self._pp_sig[0], self.rank, self.p, sa, 0, pa, len(pull), None,
                                          out_ptr if pull else None, grid_len, buf_vecs, self.epoch | ZC_TAG,
                                          self._grid(grid_len, "plan"), edev, st), "mp4x_ipc_copy_plan(zero-copy)")

    def gather_registered(self, flat: torch.Tensor, froms, tos, root: int) -> bool:
        """Root pulls every rank's ``[froms[j], tos[j])`` straight from the peers' registered
        tensors (16-byte ranges).  False (nothing done, on every rank alike) otherwise."""
        z = self._zc_segs(flat, froms, tos)
        if z is None:
            return False
        rng, peers, lo, hi = z
        ln = [h - l_ for l_, h in zip(lo, hi)]
        if max(ln) == 0:
            return True
        pull = [(lo[j], lo[j], ln[j], j) for j in range(self.p) if j != root and ln[j]] if self.rank == root else []
        self._plan_registered(peers, pull, rng.data_ptr(), max(ln), rng.numel() * rng.element_size() // 16)
        return True

    def scatter_registered(self, flat: torch.Tensor, froms, tos, root: int) -> bool:
        """Every rank pulls its ``[froms[r], tos[r])`` straight from the root's registered tensor."""
        z = self._zc_segs(flat, froms, tos)
        if z is None:
            return False
        rng, peers, lo, hi = z
        ln = [h - l_ for l_, h in zip(lo, hi)]
        if max(ln) == 0:
            return True
        r = self.rank
        pull = [(lo[r], lo[r], ln[r], root)] if r != root and ln[r] else []
        self._plan_registered(peers, pull, rng.data_ptr(), max(ln), rng.numel() * rng.element_size() // 16)
        return True

    # ---------------------------------------------------------------- RS / AG over ragged ranges
    # Results are produced inside the staging buffer (always 16-byte aligned) and copied out, so
    # whether a call qualifies depends only on the (rank-independent) ranges: every rank takes
    # the same path without an extra agreement round.
    def _range_ok(self, view: torch.Tensor, froms, tos) -> bool:
        es = view.element_size()
        base = froms[0]
        if (tos[-1] - base) * es > self.nbytes:
            return False
        return all(((f - base) * es) % 16 == 0 and ((t - base) * es) % 16 == 0 for f, t in zip(froms, tos))

    def _next_epoch(self, st, capturing=None):
        """The epoch of a launch on stream ``st`` (every IPC launch goes through here): the
        communicator's stream order first (parallel/order.py: a launch on another stream than the
        previous one waits for it), then the device counter's bump (graph mode; its address is
        returned) or the host epoch's (None)."""
        if self._epoch_dev is not None:
            self.order().enter(st)
            check(self.lib.mp4x_ipc_bump_epoch(self._epoch_dev.data_ptr(), st), "ipc_bump_epoch")
            return self._epoch_dev.data_ptr()
        if capturing if capturing is not None else torch.cuda.is_current_stream_capturing():
            raise Mp4jException("call IpcAllreduce.prepare_graph() (collectively) before capturing")
        self.order().enter(st)
        self.epoch = ((self.epoch + 1) & 0x3FFFFFFF) or 2   # (ipc.next_epoch)
        return None

    def _launch_stream(self) -> int:
        """The current stream, joined to the communicator's stream order: every staging copy,
        memset and kernel a form queues after this is ordered after the previous collective."""
        st = stream_ptr()
        self.order().enter(st)
        return st

    def order(self):
        """The stream-order guard of this instance's launches: the owning engine's (one per
        communicator, :meth:`use_order`), else one of its own."""
        o = self.__dict__.get("_order")
        if o is None:
            from .order import CommOrder
            o = self.__dict__["_order"] = CommOrder()
        return o

    def use_order(self, order) -> None:
        """Share the communicator's stream-order guard (set by the engine before any launch)."""
        self.__dict__["_order"] = order
        self.__dict__["_fast_state"] = None

    def _grid(self, nvec: int, family: str = "plan", dtype=None, op=None) -> int:
        """Explicit grid for a per-block-barrier kernel.  ``nvec`` must be RANK-INDEPENDENT (the
        largest segment of any rank): block b of every rank has to exist to meet block b of the
        peers, so ragged segments may not size the grid per rank.

        At least 8 blocks: workgroups are dealt round-robin over the 8 XCDs, so every XCD runs
        the barriers' system-scope release / acquire (each XCD has its own L2) even when the
        data would fit fewer blocks — the zero-copy forms read and write the peers' cached
        tensors.  On a shared GPU the cap of the launched kernel applies (:meth:`grid_cap`)."""
        cap = self.grid_cap(family, dtype, op)
        return max(min(8, cap), min(cap, -(-nvec // 512)))

    def reduce_scatter(self, view: torch.Tensor, froms, tos, op) -> bool:
        """In place: ``view[froms[r]:tos[r]]`` <- op over all ranks of that range (ragged ranges
        whose byte offsets are 16-byte multiples).  Returns False (nothing done) otherwise."""
        if not self._range_ok(view, froms, tos) or not self.supports(view, op):
            return False
        self.raise_if_failed()
        es = view.element_size()
        flat = view.view(-1)
        base, r = froms[0], self.rank
        st = self._launch_stream()
        n = (tos[-1] - base) * es
        if self._fuse_copy and n:
            # one launch: the kernel stages this rank's range and writes its segment in place.
            # The path depends on rank-independent facts only (ranges, env); a range that is not
            # 16-byte aligned on THIS rank goes through an aligned temporary instead.
            rng = flat[base:tos[-1]]
            tmp = None
            if rng.data_ptr() % 16:
                tmp = torch.empty(n, dtype=torch.uint8, device=view.device)
                tmp.copy_(rng.view(torch.uint8))
            b16 = tmp.data_ptr() if tmp is not None else rng.data_ptr()
            mine_off = (froms[r] - base) * es
            edev = self._next_epoch(st)
            lo_a = (c_int64 * self.p)(*[(f - base) * es // 16 for f in froms])
            hi_a = (c_int64 * self.p)(*[(t - base) * es // 16 for t in tos])
            maxv = max(h - l_ for l_, h in zip(lo_a, hi_a))
            dt, blocks = int(dtype_of_torch(view.dtype)), self._grid(maxv, "rs", view.dtype, op)
            sink = self._plan_sink
            if sink is not None:
                sink.append(("rs", dt, int(op.code), lo_a, hi_a, b16, b16 + mine_off, blocks, edev))
            check(self.lib.mp4x_ipc_reduce_scatter_from(dt, int(op.code), self._pp_data[0], self._pp_sig[0], r, self.p,
                                                        lo_a, hi_a, b16, b16 + mine_off, self.epoch, blocks, edev, st),
                  "mp4x_ipc_reduce_scatter_from")
            if tmp is not None and tos[r] > froms[r]:
                flat[froms[r]:tos[r]].view(torch.uint8).copy_(tmp[mine_off:(tos[r] - base) * es])
            return True
        if n:
            check(self.lib.mp4x_memcpy_async(self._data.value, flat[base:].data_ptr(), n, st), "ipc RS staging")
        edev = self._next_epoch(st)
        lo, hi = (froms[r] - base) * es // 16, (tos[r] - base) * es // 16
        mine = self._data.value + lo * 16          # reduced in place inside the own buffer
        maxv = max((t - f) * es // 16 for f, t in zip(froms, tos))
        check(self.lib.mp4x_ipc_reduce_scatter(int(dtype_of_torch(view.dtype)), int(op.code), self._pp_data[0],
                                               self._pp_sig[0], r, self.p, lo, hi, mine, self.epoch,
                                               self._grid(maxv, "rs", view.dtype, op), edev, st), "mp4x_ipc_reduce_scatter")
        if hi > lo:
            check(self.lib.mp4x_memcpy_async(flat[froms[r]:].data_ptr(), mine, (hi - lo) * 16, st), "ipc RS out")
        return True

    def allgather(self, view: torch.Tensor, froms, tos) -> bool:
        """In place: every rank's ``view[froms[j]:tos[j]]`` lands everywhere (ragged, 16-byte offsets)."""
        if not self._range_ok(view, froms, tos):
            return False
        self.raise_if_failed()
        es = view.element_size()
        flat = view.view(-1)
        base, r = froms[0], self.rank
        if self._fuse_copy and (not torch.cuda.is_current_stream_capturing() or self._epoch_dev is not None):
            # one copy-plan launch: stage the own segment in-kernel, pull every peer's segment
            # straight into the output (no staging copy, no copy-out).  A range that is not
            # 16-byte aligned on THIS rank runs the same plan on an aligned temporary, so every
            # rank takes the same protocol.
            lo = [(f - base) * es // 16 for f in froms]
            ln = [(t - f) * es // 16 for f, t in zip(froms, tos)]
            grid = max(ln)
            if grid == 0:
                return True
            rng = flat[base:tos[-1]]
            tmp = None
            if rng.data_ptr() % 16:
                tmp = torch.empty(rng.numel() * es, dtype=torch.uint8, device=view.device)
                tmp.copy_(rng.view(torch.uint8))
            b16 = tmp.data_ptr() if tmp is not None else rng.data_ptr()
            pulls = [(lo[j], lo[j], ln[j], j) for j in range(self.p) if j != r and ln[j]]
            self._plan([(lo[r], lo[r], ln[r], 0)] if ln[r] else [], pulls, b16, b16, grid)
            if tmp is not None:
                rng.view(torch.uint8).copy_(tmp)
            return True
        st = self._launch_stream()
        seg = (tos[r] - froms[r]) * es
        if seg:
            check(self.lib.mp4x_memcpy_async(self._data.value + (froms[r] - base) * es, flat[froms[r]:].data_ptr(),
                                             seg, st), "ipc AG staging")
        edev = self._next_epoch(st)
        lo = (c_int64 * self.p)(*[(f - base) * es // 16 for f in froms])
        hi = (c_int64 * self.p)(*[(t - base) * es // 16 for t in tos])
        maxlen = max(h - l_ for l_, h in zip(lo, hi))
        # peers' segments land in the OWN buffer (only the own segment is read remotely), then one copy out
        check(self.lib.mp4x_ipc_allgather(self._pp_data[0], self._pp_sig[0], r, self.p, lo, hi, self._data.value,
                                          self.epoch, self._grid(maxlen, "gather"), edev, st), "mp4x_ipc_allgather")
        n = (tos[-1] - base) * es
        if n:
            check(self.lib.mp4x_memcpy_async(flat[base:].data_ptr(), self._data.value, n, st), "ipc AG out")
        return True

    # ---------------------------------------------------------------- broadcast / scatter / gather
    # One copy-plan kernel per call (csrc/runtime/ipc.hip k_ipc_copy_plan): the owning ranks stage
    # their data into their own buffers inside the kernel, the receivers pull it over xGMI.  For
    # messages up to the buffer size; ranges must be whole 16-byte vectors from a 16-byte aligned
    # tensor (checked identically on every rank from the shared arguments).
    _plan_sink = None        # a list while the engine records a call's plans (latency memo)

    def _plan(self, stage, pull, src_ptr, out_ptr, grid_len) -> None:
        self.raise_if_failed()
        sa = (c_int64 * (4 * max(1, len(stage))))(*[x for it in stage for x in it])
        pa = (c_int64 * (4 * max(1, len(pull))))(*[x for it in pull for x in it])
        # every refusal BEFORE the epoch moves: a refused plan leaves this rank's epoch in step
        check(self.lib.mp4x_ipc_copy_plan_check(self.rank, self.p, sa, len(stage), pa, len(pull), src_ptr, out_ptr,
                                                self.nbytes // 16), "mp4x_ipc_copy_plan")
        st = self._launch_stream()
        edev = self._next_epoch(st)
        blocks = self._grid(grid_len)
        sink = self._plan_sink
        if sink is not None:
            sink.append(("plan", sa, len(stage), pa, len(pull), src_ptr, out_ptr, grid_len, self.nbytes // 16, blocks,
                         edev))
        check(self.lib.mp4x_ipc_copy_plan(self._pp_data[0], self._pp_sig[0], self.rank, self.p, sa, len(stage), pa,
                                          len(pull), src_ptr, out_ptr, grid_len, self.nbytes // 16, self.epoch,
                                          blocks, edev, st), "mp4x_ipc_copy_plan")

    def _vec_ok(self, view: torch.Tensor, bounds) -> bool:
        """Rank-independent qualification (shape, ranges, capture state).  The tensor's own
        address is NOT part of it: an oddly offset tensor on one rank goes through
        :meth:`_aligned` so every rank still runs the same plan."""
        es = view.element_size()
        if not view.is_contiguous():
            return False
        if torch.cuda.is_current_stream_capturing() and self._epoch_dev is None:
            return False
        return all((b * es) % 16 == 0 for b in bounds)

    @staticmethod
    def _aligned(view: torch.Tensor, fn) -> bool:
        """Run ``fn`` on an allocator-aligned copy of ``view`` and copy the result back."""
        tmp = torch.empty_like(view, memory_format=torch.contiguous_format)
        tmp.copy_(view)
        ok = fn(tmp)
        view.copy_(tmp)
        return ok

    def broadcast(self, view: torch.Tensor, frm: int, to: int, root: int) -> bool:
        es = view.element_size()
        if to <= frm or (to - frm) * es > self.nbytes or not self._vec_ok(view, (frm, to)):
            return False
        if view.data_ptr() % 16:
            return self._aligned(view, lambda t: self.broadcast(t, frm, to, root))
        base = view.data_ptr()
        L = (to - frm) * es // 16
        off = frm * es // 16
        if self.rank == root:
            self._plan([(off, 0, L, 0)], [], base, None, L)
        else:
            self._plan([], [(0, off, L, root)], None, base, L)
        return True

    def scatter(self, view: torch.Tensor, froms, tos, root: int) -> bool:
        es = view.element_size()
        p, r = self.p, self.rank
        lens = [(t - f) * es // 16 for f, t in zip(froms, tos)]
        if sum(ln for j, ln in enumerate(lens) if j != root) * 16 > self.nbytes or \
                not self._vec_ok(view, list(froms) + list(tos)):
            return False
        if view.data_ptr() % 16:
            return self._aligned(view, lambda t: self.scatter(t, froms, tos, root))
        grid = max([ln for j, ln in enumerate(lens) if j != root] or [0])
        if grid == 0:
            return True
        boff, o = [0] * p, 0
        for j in range(p):
            if j != root:
                boff[j] = o
                o += lens[j]
        base = view.data_ptr()
        if r == root:
            self._plan([(froms[j] * es // 16, boff[j], lens[j], 0) for j in range(p) if j != root], [], base, None,
                       grid)
        else:
            self._plan([], [(boff[r], froms[r] * es // 16, lens[r], root)], None, base, grid)
        return True

    def gather(self, view: torch.Tensor, froms, tos, root: int) -> bool:
        es = view.element_size()
        p, r = self.p, self.rank
        lens = [(t - f) * es // 16 for f, t in zip(froms, tos)]
        if max(lens) * 16 > self.nbytes or not self._vec_ok(view, list(froms) + list(tos)):
            return False
        if view.data_ptr() % 16:
            return self._aligned(view, lambda t: self.gather(t, froms, tos, root))
        grid = max([ln for j, ln in enumerate(lens) if j != root] or [0])
        if grid == 0:
            return True
        base = view.data_ptr()
        if r == root:
            self._plan([], [(0, froms[j] * es // 16, lens[j], j) for j in range(p) if j != root], None, base, grid)
        else:
            self._plan([(froms[r] * es // 16, 0, lens[r], 0)], [], base, None, grid)
        return True

    # ---------------------------------------------------------------- piecewise large bcast / scatter / gather
    # Any size through the buffer, one copy-plan launch per piece.  Piece i moves slab i of every
    # segment (the same per-segment slab on every rank: grids and piece counts come from the
    # shared ranges only).  The receivers pull every peer's slab at once (all links busy).
    def broadcast_large(self, view: torch.Tensor, frm: int, to: int, root: int) -> bool:
        es = view.element_size()
        if to <= frm or not self._vec_ok(view, (frm, to)):
            return False
        if view.data_ptr() % 16:
            return self._aligned(view, lambda t: self.broadcast_large(t, frm, to, root))
        base = view.data_ptr()
        L, off, s = (to - frm) * es // 16, frm * es // 16, self.nbytes // 16
        for o in range(0, L, s):
            m = min(s, L - o)
            if self.rank == root:
                self._plan([(off + o, 0, m, 0)], [], base, None, m)
            else:
                self._plan([], [(0, off + o, m, root)], None, base, m)
        return True

    def scatter_large(self, view: torch.Tensor, froms, tos, root: int) -> bool:
        es = view.element_size()
        p, r = self.p, self.rank
        if not self._vec_ok(view, list(froms) + list(tos)):
            return False
        if view.data_ptr() % 16:
            return self._aligned(view, lambda t: self.scatter_large(t, froms, tos, root))
        lens = [(t - f) * es // 16 for f, t in zip(froms, tos)]
        others = [j for j in range(p) if j != root]
        s = (self.nbytes // 16) // max(1, len(others))          # slab per segment per piece
        slot = {j: k * s for k, j in enumerate(others)}
        base = view.data_ptr()
        for i in range(-(-max([lens[j] for j in others] or [0]) // s)):
            ln = {j: max(0, min(lens[j] - i * s, s)) for j in others}
            grid = max(ln.values())
            if grid == 0:
                continue
            if r == root:
                self._plan([(froms[j] * es // 16 + i * s, slot[j], ln[j], 0) for j in others if ln[j]], [], base,
                           None, grid)
            else:
                self._plan([], [(slot[r], froms[r] * es // 16 + i * s, ln[r], root)] if ln[r] else [], None, base,
                           grid)
        return True

    def gather_large(self, view: torch.Tensor, froms, tos, root: int) -> bool:
        es = view.element_size()
        p, r = self.p, self.rank
        if not self._vec_ok(view, list(froms) + list(tos)):
            return False
        if view.data_ptr() % 16:
            return self._aligned(view, lambda t: self.gather_large(t, froms, tos, root))
        lens = [(t - f) * es // 16 for f, t in zip(froms, tos)]
        others = [j for j in range(p) if j != root]
        s = self.nbytes // 16                                    # each rank stages one slab
        base = view.data_ptr()
        for i in range(-(-max([lens[j] for j in others] or [0]) // s)):
            ln = {j: max(0, min(lens[j] - i * s, s)) for j in others}
            grid = max(ln.values())
            if grid == 0:
                continue
            if r == root:
                self._plan([], [(0, froms[j] * es // 16 + i * s, ln[j], j) for j in others if ln[j]], None, base,
                           grid)
            else:
                self._plan([(froms[r] * es // 16 + i * s, 0, ln[r], 0)] if ln[r] else [], [], base, None, grid)
        return True

    # ---------------------------------------------------------------- piecewise large RS / AG
    # Messages beyond the staging buffer (e.g. the ZeRO reduce-scatter + all-gather of a 4 GB
    # bf16 tensor, BASELINE config 3): piece i covers slab i of EVERY rank's segment, staged at
    # offset j * slab in the buffer, so the direct kernels above run unchanged per piece (all
    # links busy, fused peer-load + reduce for RS).  Segments must be whole 16-byte vectors.
    def _slab(self, es: int) -> int:
        """Elements of each rank's segment per piece (a 16-byte multiple)."""
        return (self.nbytes // self.p) // 16 * 16 // es

    def large_ok(self, view: torch.Tensor, froms, tos) -> bool:
        es = view.element_size()
        if self._slab(es) <= 0 or not view.is_contiguous():
            return False
        if torch.cuda.is_current_stream_capturing() and self._epoch_dev is None:
            return False
        return all(((t - f) * es) % 16 == 0 for f, t in zip(froms, tos))

    def reduce_scatter_large(self, view: torch.Tensor, froms, tos, op) -> bool:
        """In place ``view[froms[r]:tos[r]]`` <- op over all ranks, any message size, in pieces."""
        if not self.supports(view, op) or not self.large_ok(view, froms, tos):
            return False
        self.raise_if_failed()
        es = view.element_size()
        flat = view.view(-1)
        p, r = self.p, self.rank
        counts = [t - f for f, t in zip(froms, tos)]
        s = self._slab(es)
        sv = s * es // 16
        buf = self._data.value
        dt = int(dtype_of_torch(view.dtype))
        st = self._launch_stream()
        for i in range(-(-max(counts) // s)):
            lens = [max(0, min(c - i * s, s)) for c in counts]
            for j in range(p):
                if lens[j]:
                    check(self.lib.mp4x_memcpy_async(buf + j * s * es, flat[froms[j] + i * s:].data_ptr(), lens[j] * es,
                                                     st), "ipc RS-large staging")
            edev = self._next_epoch(st)
            lo = r * sv
            hi = lo + lens[r] * es // 16
            check(self.lib.mp4x_ipc_reduce_scatter(dt, int(op.code), self._pp_data[0], self._pp_sig[0], r, p, lo, hi,
                                                   buf + lo * 16, self.epoch,
                                                   self._grid(max(lens) * es // 16, "rs", view.dtype, op), edev,
                                                   st), "mp4x_ipc_reduce_scatter")
            if lens[r]:
                check(self.lib.mp4x_memcpy_async(flat[froms[r] + i * s:].data_ptr(), buf + lo * 16, lens[r] * es, st),
                      "ipc RS-large out")
        return True

    def allgather_large(self, view: torch.Tensor, froms, tos) -> bool:
        """In place: every rank's ``view[froms[j]:tos[j]]`` lands everywhere, any size, in pieces."""
        if not self.large_ok(view, froms, tos):
            return False
        self.raise_if_failed()
        es = view.element_size()
        flat = view.view(-1)
        p, r = self.p, self.rank
        counts = [t - f for f, t in zip(froms, tos)]
        s = self._slab(es)
        sv = s * es // 16
        buf = self._data.value
        st = self._launch_stream()
        for i in range(-(-max(counts) // s)):
            lens = [max(0, min(c - i * s, s)) for c in counts]
            if lens[r]:
                check(self.lib.mp4x_memcpy_async(buf + r * s * es, flat[froms[r] + i * s:].data_ptr(), lens[r] * es,
                                                 st), "ipc AG-large staging")
            edev = self._next_epoch(st)
            lo = (c_int64 * p)(*[j * sv for j in range(p)])
            hi = (c_int64 * p)(*[j * sv + lens[j] * es // 16 for j in range(p)])
            check(self.lib.mp4x_ipc_allgather(self._pp_data[0], self._pp_sig[0], r, p, lo, hi, buf, self.epoch,
                                              self._grid(max(lens) * es // 16, "gather"), edev, st),
                  "mp4x_ipc_allgather")
            for j in range(p):
                if j != r and lens[j]:
                    check(self.lib.mp4x_memcpy_async(flat[froms[j] + i * s:].data_ptr(), buf + j * s * es,
                                                     lens[j] * es, st), "ipc AG-large out")
        return True
