"""Schedule autotuning of the device engine (mixin of :class:`~mp4x.parallel.device_engine.DeviceEngine`).

Every tuner times the applicable schedules of one collective on a scratch tensor, checks each
candidate first against an exact pattern (a wrong schedule is never pinned), takes the MAX
time over ranks (so every rank pins the same schedule) and pins the fastest per
(dtype, op, ceil-log2 size) class: allreduce (RCCL, RCCL with more channels, IPC one-/two-shot,
pipelined, zero-copy pull / push and their grid variants, a2a, rhd, node-aware), reduce-scatter /
all-gather, and the rooted reduce / broadcast / gather / scatter.  The pinned table persists
(``MP4X_TUNE_FILE``) and is shared from rank 0.  The reference has no counterpart: its schedule
is fixed per collective (ring RS + AG, trees; /root/reference/README.md:286-294).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..exceptions import Mp4jException
from ..operators import OpCode
from ..ops.native import capturing_now
from ..utils.commutils import CommUtils

LOG = logging.getLogger("mp4x.device")


def _tune_key(dtype, op, nbytes: int) -> tuple:
    return (dtype, int(op.code), max(0, int(nbytes) - 1).bit_length())   # ceil(log2(nbytes))


# Grid variants of the zero-copy two-shot the allreduce autotuner tries on a GPU of its own
# (``ipc2z_b<N>``: N blocks instead of up to one per CU).  How many concurrent readers keep 7
# xGMI links busy without thrashing the remote request queues is a property of the topology,
# so it is measured, not assumed.
ZC_GRIDS = (64, 128)


def zc_grid(algo: str):
    """(base schedule, grid) of an allreduce schedule name: ``ipc2z_b64`` -> (``ipc2z``, 64)."""
    if algo.startswith("ipc2z_b") and algo[7:].isdigit():
        return "ipc2z", int(algo[7:])
    return algo, 0


class _TunedTable(dict):
    """The pinned-schedule table; ``gen`` counts its mutations, so :meth:`DeviceEngine.select`
    can memoise its decisions and still see every re-tune, table load or clear."""
    gen = 0
    on_change = None          # the engine's latency-memo invalidation

    def _bump(self):
        self.gen += 1
        if self.on_change is not None:
            self.on_change()

    def __setitem__(self, k, v):
        self._bump()
        super().__setitem__(k, v)

    def __delitem__(self, k):
        self._bump()
        super().__delitem__(k)

    def pop(self, *a):
        self._bump()
        return super().pop(*a)

    def popitem(self):
        self._bump()
        return super().popitem()

    def clear(self):
        self._bump()
        super().clear()

    def update(self, *a, **k):
        self._bump()
        super().update(*a, **k)

    def pinned(self, key: tuple):
        """The schedule for ``key`` = (..., size class): the pin of that class, else — between two
        measured classes of the same (kind, dtype, op) that pinned the SAME schedule — that
        schedule (it won on both sides; the tier sweep visits 4 KiB, 64 KiB, 256 KiB, ... so the
        classes in between follow the measurements instead of the model defaults), else None."""
        hit = self.get(key)
        if hit is not None or not self:
            return hit
        pre, cls = key[:-1], key[-1]
        lo = hi = None
        for k, v in self.items():
            if len(k) != len(key) or k[:-1] != pre:
                continue
            c = k[-1]
            if c < cls and (lo is None or c > lo[0]):
                lo = (c, v)
            elif c > cls and (hi is None or c < hi[0]):
                hi = (c, v)
        return lo[1] if lo is not None and hi is not None and lo[1] == hi[1] else None

    def setdefault(self, k, d=None):
        self._bump()
        return super().setdefault(k, d)


_DIAG = os.environ.get("MP4X_AUTOTUNE_DIAG", "0") == "1"


def _diag_mismatch(rank: int, name: str, got: torch.Tensor, exp: torch.Tensor) -> None:
    """``MP4X_AUTOTUNE_DIAG=1``: what a wrong probe result holds (stderr, one line per rank): the
    count, the first mismatches (index, got, expected) and how many wrong elements are the probe's
    fill (-1), zero, or another rank's pattern value."""
    import sys
    bad = (got != exp).nonzero().flatten()
    if bad.numel() == 0:
        return
    g, e = got[bad], exp[bad]
    first = [(int(i), float(a), float(b)) for i, a, b in zip(bad[:6].tolist(), g[:6].tolist(), e[:6].tolist())]
    print(f"[autotune-diag] rank {rank} {name}: {bad.numel()} of {got.numel()} wrong; first {first}; "
          f"fill(-1) {int((g == -1).sum())}, zero {int((g == 0).sum())}, "
          f"span [{int(bad[0])}, {int(bad[-1])}]", file=sys.stderr, flush=True)


class AutotuneMixin:
    """The tuners, probes and the persisted table; state lives on the engine."""

    # ------------------------------------------------------------------ autotuning
    def _algo_valid(self, algo: str, op, dtype, nbytes: int) -> bool:
        if algo == "rccl":
            return self.rccl_ok(op, dtype)
        if algo.startswith("rccl_c"):
            return self.backend == "nccl" and self.rccl_ok(op, dtype)
        if algo == "hier":
            return self._hier_ok(op, dtype, nbytes)
        if zc_grid(algo)[0] in ("ipc1", "ipc2", "ipc2p", "ipc2z", "ipc2w"):
            return self._ipc_ok(op, dtype, nbytes)
        if algo == "rhd":
            return not getattr(op, "is_custom", False)
        return algo == "a2a"

    def _stand_in(self) -> bool:
        """gloo standing in for RCCL on GPU tensors (the one-GPU rehearsals): its device paths stage
        through host memory and, with 4-8 processes on one GPU, leave every later barrier kernel
        time-sliced (~70-100 ms per call at any size, profiles/r3/round/rehearsal_np8.jsonl), so
        the autotuners skip the transport candidates when IPC ones exist
        (``MP4X_AUTOTUNE_GLOO=1`` keeps them).  Never true with RCCL underneath."""
        return self.backend == "gloo" and self.device.type == "cuda" and self.ipc_enabled and \
            os.environ.get("MP4X_AUTOTUNE_GLOO", "0") != "1"

    @staticmethod
    def _extra_schedules() -> bool:
        """``MP4X_AUTOTUNE_EXTRA=1``: the opt-in schedules join the autotune candidates (RCCL with
        pinned channel counts, the pipelined staged two-shot, the zero-copy grid variants, rhd,
        the composite broadcast).  Off by default: every schedule tried on first contact with a
        topology is a risk and costs tuning time; each stays reachable by
        name (``MP4X_DEVICE_ALGO``, ``MP4X_AUTOTUNE_CANDIDATES``, a tune file)."""
        return os.environ.get("MP4X_AUTOTUNE_EXTRA", "0") == "1"

    def allreduce_candidates(self, nbytes: int, op, dtype) -> List[str]:
        """The default decision tree's allreduce candidates (DESIGN.md "Default schedules"): at
        most six — ``rccl``, ``ipc1`` (<= 4 MiB), ``ipc2``, ``ipc2z``, ``ipc2w``, ``a2a``.  The rest only
        with :meth:`_extra_schedules`; ``hier`` (a multi-node job) also with ``MP4X_HIER=1``."""
        c = []
        extra = self._extra_schedules()
        if self._stand_in() and self._ipc_ok(op, dtype, nbytes):
            return (["ipc1"] if nbytes <= (4 << 20) else []) + ["ipc2"] + \
                (["ipc2p"] if extra and nbytes > self.ipc_twoshot_max else []) + \
                (["ipc2z", "ipc2w"] if self._zc else [])
        if self.rccl_ok(op, dtype):
            c.append("rccl")
            if extra and self.backend == "nccl" and nbytes >= (64 << 20):
                c += [f"rccl_c{n}" for n in self.RCCL_CTA_VARIANTS]
        if self._ipc_ok(op, dtype, nbytes) and self.device.type == "cuda":
            if nbytes <= (4 << 20):
                c.append("ipc1")
            c.append("ipc2")
            if extra and nbytes > self.ipc_twoshot_max:
                c.append("ipc2p")     # pipelined pieces: input copies overlap the xGMI-bound kernel
            if self._zc:
                c.append("ipc2z")     # zero-copy two-shot on a registered tensor (one kernel)
                c.append("ipc2w")     # ... its push form: every xGMI transfer a posted write
                if extra and nbytes >= (64 << 20) and not getattr(self._ipc_obj, "shared_gpu", True):
                    c += [f"ipc2z_b{g}" for g in ZC_GRIDS]     # ... with fewer, longer-lived blocks
        if (extra or self._hier_auto) and self._hier_ok(op, dtype, nbytes):
            c.append("hier")          # opt-in: multi-node only (one node is the whole target machine)
        c.append("a2a")
        if extra and nbytes <= (64 << 20):
            c.append("rhd")
        return c

    def autotune_allreduce(self, like: torch.Tensor, operator, candidates: Optional[Sequence[str]] = None,
                           iters: int = 3) -> Dict[str, float]:
        """Time every applicable allreduce schedule on a scratch tensor shaped like ``like`` and
        pin the fastest for this (dtype, op, size class).  Collective: every rank calls it with
        the same shape; the decision uses the MAX time over ranks, so all ranks agree.

        Returns {algo: seconds per call} (inf for a schedule that failed on any rank)."""
        # a scratch tensor for this tune only: registered for the zero-copy candidates, deregistered
        # and dropped afterwards (nothing is retained per size class; its memory goes back to the
        # caching allocator and a re-tune of the class usually gets the same block again)
        view = torch.zeros(like.numel(), dtype=like.dtype, device=like.device)
        op = self._op(operator, view)
        nbytes = view.numel() * view.element_size()
        if candidates is None and os.environ.get("MP4X_AUTOTUNE_CANDIDATES"):
            candidates = [c.strip() for c in os.environ["MP4X_AUTOTUNE_CANDIDATES"].split(",") if c.strip()]
        cands = [c for c in (candidates or self.allreduce_candidates(nbytes, op, view.dtype))
                 if self._algo_valid(c, op, view.dtype, nbytes)]
        times = []
        if self.watchdog is not None:
            self.watchdog.paused += 1     # IPC timeouts here are expected probe results, not failures
        registered = False
        try:
            with self.probing():
                try:
                    if any(zc_grid(c)[0] in ("ipc2z", "ipc2w") for c in cands):
                        registered = self.register_buffer(view)     # collective; False on every rank alike
                        if not registered or (self._ipc_obj.scratch_of(view) is None and "ipc2w" in cands):
                            # (the push form needs every rank's scratch: agreed inside register)
                            cands[:] = [c for c in cands if c != "ipc2w" or registered and
                                        self._ipc_obj.scratch_of(view) is not None]
                        if not registered:
                            cands[:] = [c for c in cands if zc_grid(c)[0] not in ("ipc2z", "ipc2w")]
                    for c in cands:
                        times.append(self._time_candidate(c, view, op, iters))
                finally:
                    if registered:
                        self.deregister_buffer(view)        # collective, ordered (ipc.deregister)
        finally:
            if self.watchdog is not None:
                self.watchdog.paused -= 1
        tt = torch.tensor(times, dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        self.coll.all_reduce(tt, OpCode.MAX)
        res = dict(zip(cands, tt.cpu().tolist()))
        best = min(res, key=res.get) if res else None
        if best is not None and res[best] != float("inf"):
            self._tuned[_tune_key(view.dtype, op, nbytes)] = best
            self._autosave()
        return res

    def autotune_reduce_scatter(self, like: torch.Tensor, operator, iters: int = 3) -> Dict[str, float]:
        """Reduce-scatter twin of :meth:`autotune_allreduce` (equal split of ``like``): times RCCL
        ``reduce_scatter_tensor``, the piecewise IPC kernels and the a2a schedule, MAX over ranks,
        and pins the fastest for this (dtype, op, size class).  Collective."""
        view = torch.zeros(like.numel(), dtype=like.dtype, device=like.device)
        op = self._op(operator, view)
        froms, tos, _ = CommUtils.even_split(0, view.numel(), self.p)
        cands = ["rccl", "a2a"] + (["ipc"] if self.ipc_enabled and self._ipc_ok(op, view.dtype, 16) else [])
        if self._stand_in() and "ipc" in cands:
            cands = ["ipc"]
        r = self.rank

        def probe():
            exp = self._fill_probe(view, op)
            if exp is None:
                return None

            def check():
                bad = int((view[froms[r]:tos[r]] != exp[froms[r]:tos[r]]).sum())
                view.zero_()
                return bad
            return check
        return self._autotune_kind("reduce_scatter", view, op, cands,
                                   lambda: self.reduce_scatter(view, froms, tos, op), iters, probe)

    def autotune_allgather(self, like: torch.Tensor, iters: int = 3) -> Dict[str, float]:
        """All-gather twin of :meth:`autotune_allreduce` (equal split): RCCL
        ``all_gather_into_tensor`` vs the piecewise IPC kernels vs grouped p2p.  Collective."""
        view = torch.zeros(like.numel(), dtype=like.dtype, device=like.device)
        froms, tos, _ = CommUtils.even_split(0, view.numel(), self.p)
        cands = ["rccl", "p2p"] + (["ipc"] if self.ipc_enabled else [])
        if self._stand_in():
            cands = ["ipc"]

        def probe():
            # owner j's segment holds i % 97 + j; after the call every rank holds every segment
            idt = torch.int32 if view.numel() < (1 << 31) else torch.int64
            exp = torch.arange(view.numel(), device=view.device, dtype=idt).remainder_(97)
            for j in range(self.p):
                exp[froms[j]:tos[j]] += j
            exp = exp.to(view.dtype)
            view.fill_(-1)
            view[froms[self.rank]:tos[self.rank]] = exp[froms[self.rank]:tos[self.rank]]

            def check():
                bad = int((view != exp).sum())
                view.zero_()
                return bad
            return check
        return self._autotune_kind("allgather", view, None, cands, lambda: self.allgather(view, froms, tos), iters,
                                   probe)

    def _autotune_kind(self, kind: str, view: torch.Tensor, op, cands, run, iters: int,
                       probe=None, pin_rccl: bool = False) -> Dict[str, float]:
        """``pin_rccl``: the kind's default path is not plain RCCL at every size (reduce /
        broadcast / gather / scatter take IPC tiers below the two-shot size), so RCCL is timed and
        pinned explicitly as the schedule ``rccl`` instead of as "nothing pinned"."""
        key = self._rsag_key(kind, view, op)
        times = []
        if self.watchdog is not None:
            self.watchdog.paused += 1
        try:
            with self.probing():
                self._autotune_loop(kind, view, cands, run, iters, probe, pin_rccl, key, times)
        finally:
            self._tuned.pop(key, None)
            if self.watchdog is not None:
                self.watchdog.paused -= 1
        tt = torch.tensor(times, dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        self.coll.all_reduce(tt, OpCode.MAX)
        res = dict(zip(cands, tt.cpu().tolist()))
        best = min(res, key=res.get) if res else None
        if best is not None and (best != "rccl" or pin_rccl) and res[best] != float("inf"):
            self._tuned[key] = best
        self._autosave()
        return res

    def _autotune_loop(self, kind, view, cands, run, iters, probe, pin_rccl, key, times) -> None:
        for c in cands:
            if c == "rccl" and not pin_rccl:
                self._tuned.pop(key, None)
            else:
                self._tuned[key] = c
            times.append(self._time_fn(run, uses_ipc=c not in ("rccl", "p2p"), iters=iters,
                                       name=f"{kind}:{c}", probe=probe))

    # ------------------------------------------------------------------ reduce / broadcast / gather / scatter
    def _root_tuned(self, kind: str, view: torch.Tensor, op) -> Optional[str]:
        """Schedule pinned by the autotuners below for this (kind, dtype, op, size class), or
        None.  Only for unforced, uncaptured calls (a capture keeps the tier logic)."""
        if not self._tuned or self.algo not in ("", "auto") or (view.is_cuda and capturing_now()):
            return None
        return self._tuned.pinned(self._rsag_key(kind, view, op))

    def autotune_reduce(self, like: torch.Tensor, operator, root: int = 0, iters: int = 3) -> Dict[str, float]:
        """``reduce`` schedules timed side by side (RCCL ``ncclReduce``; ``ipc`` = the IPC two-shot
        allreduce, whose result every rank gets — the reduce contract leaves non-root results
        unspecified, ProcessCommSlave.java:1390-1421; ``a2a`` = reduce-scatter + gather, the
        reference's own composition), exact-probed at the root, MAX over ranks, fastest pinned
        for this (dtype, op, size class).  Collective."""
        view = torch.zeros(like.numel(), dtype=like.dtype, device=like.device)
        op = self._op(operator, view)
        nb = view.numel() * view.element_size()
        cands = (["rccl"] if self.rccl_ok(op, view.dtype) else []) + ["a2a"]
        if self.ipc_enabled and self._ipc_ok(op, view.dtype, nb):
            cands = ["ipc"] if self._stand_in() else cands + ["ipc"]
        n = view.numel()

        def probe():
            exp = self._fill_probe(view, op)
            if exp is None:
                return None

            def check():
                bad = int((view != exp).sum()) if self.rank == root else 0
                if bad and _DIAG:
                    _diag_mismatch(self.rank, "reduce", view, exp)
                view.zero_()
                return bad
            return check
        return self._autotune_kind("reduce", view, op, cands, lambda: self.reduce(view, 0, n, op, None, root), iters,
                                   probe, pin_rccl=True)

    def _copy_probe(self, view: torch.Tensor, owners):
        """Probe for the data-movement kinds: element i holds ``i % 97 + owner(i)`` where
        ``owners`` = [(from, to, rank)] says which rank's data each range is; the caller fills
        what this rank owns before the call."""
        idt = torch.int32 if view.numel() < (1 << 31) else torch.int64
        exp = torch.arange(view.numel(), device=view.device, dtype=idt).remainder_(97)
        for f, t, j in owners:
            exp[f:t] += j
        return exp.to(view.dtype)

    def autotune_broadcast(self, like: torch.Tensor, root: int = 0, iters: int = 3) -> Dict[str, float]:
        """``broadcast``: RCCL ``ncclBroadcast`` vs the piecewise IPC copy plan (every receiver
        pulls from the root over its own link) vs ``composite`` (scatter + all-gather, the
        reference's van de Geijn schedule, ProcessCommSlave.java:750-775).  Collective."""
        view = torch.zeros(like.numel(), dtype=like.dtype, device=like.device)
        n = view.numel()
        cands = ["rccl"] + (["composite"] if self._extra_schedules() else []) + \
            (["ipc"] if self.ipc_enabled and view.is_cuda else [])
        if self._stand_in():
            cands = ["ipc"]

        def probe():
            exp = self._copy_probe(view, [(0, n, root)])
            view.copy_(exp) if self.rank == root else view.fill_(-1)

            def check():
                bad = int((view != exp).sum())
                if bad and _DIAG:
                    _diag_mismatch(self.rank, "broadcast", view, exp)
                view.zero_()
                return bad
            return check
        return self._autotune_kind("broadcast", view, None, cands, lambda: self.broadcast(view, 0, n, root), iters,
                                   probe, pin_rccl=True)

    def _autotune_gs(self, kind: str, like: torch.Tensor, root: int, iters: int) -> Dict[str, float]:
        view = torch.zeros(like.numel(), dtype=like.dtype, device=like.device)
        froms, tos, _ = CommUtils.even_split(0, view.numel(), self.p)
        cands = ["p2p"] + (["ipc"] if self.ipc_enabled and view.is_cuda else [])
        if self._stand_in():
            cands = ["ipc"]
        r = self.rank

        def probe():
            exp = self._copy_probe(view, [(froms[j], tos[j], j) for j in range(self.p)])
            view.fill_(-1)
            if kind == "gather":
                view[froms[r]:tos[r]] = exp[froms[r]:tos[r]]
            elif r == root:
                view.copy_(exp)

            def check():
                if kind == "gather":
                    bad = int((view != exp).sum()) if r == root else 0
                    if bad and _DIAG:
                        _diag_mismatch(r, "gather", view, exp)
                else:
                    bad = int((view[froms[r]:tos[r]] != exp[froms[r]:tos[r]]).sum())
                    if bad and _DIAG:
                        _diag_mismatch(r, "scatter", view[froms[r]:tos[r]], exp[froms[r]:tos[r]])
                view.zero_()
                return bad
            return check
        fn = (lambda: self.gather(view, froms, tos, root)) if kind == "gather" else \
            (lambda: self.scatter(view, froms, tos, root))
        return self._autotune_kind(kind, view, None, cands, fn, iters, probe, pin_rccl=True)

    def autotune_gather(self, like: torch.Tensor, root: int = 0, iters: int = 3) -> Dict[str, float]:
        """``gather`` (even split): grouped p2p (``ncclRecv`` x p-1 at the root) vs the
        piecewise IPC copy plan (the root pulls every segment over its links).  Collective."""
        return self._autotune_gs("gather", like, root, iters)

    def autotune_scatter(self, like: torch.Tensor, root: int = 0, iters: int = 3) -> Dict[str, float]:
        """``scatter`` (even split): grouped p2p vs the piecewise IPC copy plan.  Collective."""
        return self._autotune_gs("scatter", like, root, iters)

    def _time_fn(self, run, uses_ipc: bool, iters: int, name: str, probe=None) -> float:
        """Seconds per call of ``run`` (inf when it failed or was wrong on ANY rank).  Collective.

        ``probe()`` (optional) fills the operand with an exact pattern and returns a function
        that counts wrong elements after the warm-up call (see :meth:`_fill_probe`).

        Every rank joins the same agreement collectives whatever happened locally (a local
        exception only sets a flag), so a schedule that fails on one rank cannot pair mismatched
        collectives.  Bounded: when the agreed warm-up took longer than ``MP4X_AUTOTUNE_CAP_S``
        (default 2 s) the warm-up time is the estimate and no timed calls run; otherwise the
        timed calls are capped to about that wall time."""
        cap = float(os.environ.get("MP4X_AUTOTUNE_CAP_S", "2"))
        failed, wrong, warm = 0, 0, float("inf")
        check = None
        try:
            check = probe() if probe is not None and self._verify_autotune else None
            t0 = time.perf_counter()
            run()                                # warm-up (lazy IPC / RCCL setup)
            self._sync()
            warm = time.perf_counter() - t0
            wrong = check() if check is not None else 0
        except Exception as e:       # noqa: BLE001 — a failed candidate is just not chosen
            LOG.warning("autotune: %s failed on rank %d: %s", name, self.rank, e)
            failed = 1
        timeout = self._ipc_error_flag() if uses_ipc else 0
        warm_us = int(min(warm, 1e9) * 1e6)
        local = [failed, timeout, wrong, warm_us]
        failed, timeout, nwrong, warm_us = self._agree(local)
        if _DIAG and (failed or timeout or nwrong):
            import sys
            print(f"[autotune-diag] rank {self.rank} {name}: local [failed, timeout, wrong, warm_us] {local} -> "
                  f"agreed {[failed, timeout, nwrong, warm_us]}", file=sys.stderr, flush=True)
        second = getattr(check, "second", None) if not (failed or timeout or nwrong) else None
        if second is not None:     # agreed: every rank runs the second probe call together
            try:
                check2 = second()
                run()
                self._sync()
                wrong = check2()
            except Exception as e:   # noqa: BLE001
                LOG.warning("autotune: %s failed on rank %d: %s", name, self.rank, e)
                failed = 1
            timeout = self._ipc_error_flag() if uses_ipc else 0
            failed, timeout, nwrong = self._agree([failed, timeout, wrong])
        if failed or timeout or nwrong:
            if self.rank == 0:
                LOG.warning("autotune: %s ruled out (%s)", name, "failed" if failed else
                            "IPC barrier timeout" if timeout else f"up to {nwrong} wrong elements on the probe")
            return float("inf")
        warm = warm_us / 1e6
        if warm > cap:
            return warm                          # too slow to matter: not worth timed calls
        n = max(1, min(max(1, iters), int(cap / max(warm, 1e-6))))
        dt = float("inf")
        failed = 0
        try:
            self.barrier()
            t0 = time.perf_counter()
            for _ in range(n):
                run()
            self._sync()
            dt = (time.perf_counter() - t0) / n
        except Exception as e:       # noqa: BLE001
            LOG.warning("autotune: %s failed on rank %d: %s", name, self.rank, e)
            failed = 1
        failed, timeout = self._agree([failed, self._ipc_error_flag() if uses_ipc else 0])
        return float("inf") if failed or timeout else dt

    def _ipc_error_flag(self) -> int:
        try:
            return self._ipc_error_local()
        except Exception:   # noqa: BLE001
            return 1

    # ------------------------------------------------------------------ persisted tuning table
    _KNOWN_ALGOS = {"allreduce": {"rccl", "rccl_c64", "rccl_c112", "ipc1", "ipc2", "ipc2p", "ipc2z", "ipc2w", "a2a",
                                  "rhd", "hier"} | {f"ipc2z_b{g}" for g in ZC_GRIDS},
                    "reduce_scatter": {"ipc", "a2a"}, "allgather": {"ipc", "p2p"},
                    "reduce": {"rccl", "ipc", "a2a"}, "broadcast": {"rccl", "ipc", "composite"},
                    "gather": {"p2p", "ipc"}, "scatter": {"p2p", "ipc"}}

    _topo_agreed = None

    def _topology(self) -> dict:
        """The topology a tuning table applies to: rank count, device name, backend, node count and
        the xGMI pair map of the ranks' devices (parallel/tiers.py).  Agreed at engine creation
        (rank 0's record, ``_load_shared_tuning``) so every rank keys and checks tables alike."""
        if self._topo_agreed is not None:
            return self._topo_agreed
        dev = torch.cuda.get_device_name(self.device) if self.device.type == "cuda" else "cpu"
        top = {"p": self.p, "device": dev, "backend": self.backend}
        if self.layout.multi_node:
            top["nodes"] = len(self.layout.nodes)
        if self.device.type == "cuda":
            from .tiers import xgmi_map
            top["xgmi"] = xgmi_map(self.p, self.device.index)
        return top

    def tuning_table(self) -> dict:
        """The schedules pinned by the autotuners, JSON-able, with the topology they were measured
        on (rank count, device, backend).  A table only applies to the same topology."""
        rows = []
        for k, v in sorted(self._tuned.items(), key=lambda kv: str(kv[0])):
            kind, dt, code, cls = k if isinstance(k[0], str) else ("allreduce",) + tuple(k)
            rows.append({"kind": kind, "dtype": str(dt).replace("torch.", ""), "op": int(code),
                         "size_class": int(cls), "algo": v})
        return {"topology": self._topology(), "rows": rows}

    def save_tuning(self, path: str) -> None:
        """Rank 0 writes :meth:`tuning_table` to ``path`` (atomic rename); other ranks no-op."""
        if self.rank != 0:
            return
        import json
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = f"{path}.tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(self.tuning_table(), f, indent=1)
        os.replace(tmp, path)

    def load_tuning(self, src) -> int:
        """Pin the schedules of a saved table (path or dict).  Refuses a table measured on another
        topology; skips rows naming unknown schedules.  Every rank must load the same table (a
        shared file), so the choices stay rank-consistent.  Returns the number of rows pinned."""
        import json
        table = src
        if not isinstance(src, dict):
            with open(src) as f:
                table = json.load(f)
        if table.get("topology") != self._topology():
            raise Mp4jException(f"tuning table for {table.get('topology')}, this job is {self._topology()}")
        n = 0
        for row in table.get("rows", []):
            kind, algo = row["kind"], row["algo"]
            if algo not in self._KNOWN_ALGOS.get(kind, ()):
                continue
            dt = getattr(torch, row["dtype"])
            key = (dt, int(row["op"]), int(row["size_class"]))
            self._tuned[key if kind == "allreduce" else (kind,) + key] = algo
            n += 1
        return n

    def tune_path(self):
        """Where this job's pinned table is saved: ``MP4X_TUNE_FILE``, else with
        ``MP4X_TUNE_AUTO=1`` the topology-keyed file in ``MP4X_TUNE_DIR`` (parallel/tiers.py)."""
        path = os.environ.get("MP4X_TUNE_FILE")
        if not path:
            from . import tiers
            if tiers.auto_enabled():
                path = tiers.tune_path(self._topology())
        return path

    def _autosave(self) -> None:
        path = self.tune_path()
        if path:
            try:
                self.save_tuning(path)
            except OSError as e:
                LOG.warning("could not save the tuning table to %s: %s", path, e)

    def _time_candidate(self, c: str, view: torch.Tensor, op, iters: int) -> float:
        """Seconds per call of allreduce schedule ``c`` (inf when it failed or was wrong on any
        rank; bounded, see :meth:`_time_fn`).  Collective.  The warm-up doubles as a correctness
        probe: a schedule whose result differs from the exact answer (e.g. a peer-visibility bug
        on some topology) is never pinned."""
        def probe():
            expect = self._fill_probe(view, op)
            if expect is None:
                return None

            def check():
                return int((view != expect).sum())

            def second():
                # second call straight on the first call's RESULT (as in a training loop): a
                # schedule that leaves stale cache lines of the previous call behind on this
                # topology shows here.  SUM multiplies the values p-fold (exact for wide
                # dtypes); MAX / MIN are idempotent; narrow dtypes refill a shifted pattern.
                if op.code in (OpCode.MAX, OpCode.MIN):
                    exp2 = expect
                elif view.dtype in (torch.float32, torch.float64, torch.int32, torch.int64):
                    exp2 = expect * self.p
                else:
                    exp2 = self._fill_probe(view, op, salt=1)

                def check2():
                    bad = int((view != exp2).sum())
                    view.zero_()
                    return bad
                return check2
            check.second = second
            return check
        return self._time_fn(lambda: self._run_allreduce(c, view, op), c.startswith("ipc"), iters, c, probe)

    def _ipc_error_local(self) -> int:
        mine = 0
        for inst in (self._ipc_obj, self._ipc_large, self._ipc_fp8_big):
            # read-and-clear: a candidate that timed out must not poison the next one's check
            if inst is not None and inst.error_word(clear=True):
                mine = 1
        return mine

    def _agree(self, flags: List[int]) -> List[int]:
        """Element-wise MAX of small integer flags over all ranks (collective)."""
        t = torch.tensor(flags, dtype=torch.int64, device=self.device if self.backend == "nccl" else "cpu")
        self.coll.all_reduce(t, OpCode.MAX)
        return [int(v) for v in t.tolist()]

    def _ipc_error(self) -> bool:
        """Did any IPC barrier on ANY rank time out?  (Collective: MAX of the error words.)"""
        return bool(self._agree([self._ipc_error_local()])[0])

    _verify_autotune = os.environ.get("MP4X_AUTOTUNE_VERIFY", "1") != "0"

    def _fill_probe(self, view: torch.Tensor, op, salt: int = 0) -> Optional[torch.Tensor]:
        """Fill ``view`` with this rank's probe pattern ``(i + salt) % m + (rank & 1)`` and return
        the exact allreduce of every rank's pattern (None for ops without a closed form).  Values
        stay small integers (``p * m <= ~100``), so every schedule's result is exact in any order
        and for every dtype down to int8 / bf16: the comparison is bit-exact.  A second probe with
        another ``salt`` catches a schedule that reads stale copies of the previous call's data."""
        if op.code not in (OpCode.SUM, OpCode.MAX, OpCode.MIN) or getattr(op, "is_custom", False):
            return None
        m = max(2, min(16, 100 // self.p))
        idt = torch.int32 if view.numel() < (1 << 31) else torch.int64
        base = torch.arange(salt, view.numel() + salt, device=view.device, dtype=idt).remainder_(m)
        odd = sum(r & 1 for r in range(self.p))
        view.copy_(base + (self.rank & 1))
        if op.code == OpCode.SUM:
            exp = base * self.p + odd
        elif op.code == OpCode.MAX:
            exp = base + (1 if odd else 0)
        else:
            exp = base + (0 if odd < self.p else 1)
        return exp.to(view.dtype)
