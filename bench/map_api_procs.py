#!/usr/bin/env python3
"""BASELINE config 4 with REAL processes: ``ProcessCommSlave.allreduceMap`` of a
``Dict[str, Tensor]`` (200k keys x float[64] per rank, half shared) with p processes, one
``ProcessCommSlave`` each — the deployment shape (one process per GPU), unlike
``bench/map_api.py`` whose p virtual ranks share one interpreter and one GIL.

On a one-GPU box every process uses ``cuda:0`` and gloo stands in for RCCL in the exchange
(``MP4X_DEVICE_BACKEND=gloo``: device tensors staged through host memory), so the
``exchange_and_kernels`` phase is NOT an xGMI number.  The host phases are what a rank pays
per call whatever the transport:

* ``walk_only_ms`` — the native dict walk alone (part of the agreement round below);
* ``agree_ms``  — the device/host agreement round through the control plane, which also runs
  the native dict walk (csrc/pyext/map_ext.cpp) and carries unseen keys (none in steady state);
* ``to_tensors_ms`` — dict -> (ids, rows): the walk's rows gathered with one K3 launch;
* ``exchange_and_kernels_ms`` — K4b partition, all-to-all, K5 reduce-by-key, all-gather-v;
* ``to_dict_ms`` — the lazy ``TensorMap`` result.

Reference: ProcessCommSlave.allreduceMap (J/comm/ProcessCommSlave.java:2053-2088).
  python bench/map_api_procs.py [--p 4] [--keys 200000] [--dim 64] [--iters 5] [--fresh-dict]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def body(comm, nkeys, dim, iters, fresh):
    import torch
    from mp4x import Operands, Operators
    from mp4x.parallel import sparse

    r, p = comm.getRank(), comm.getSlaveNum()
    dev = torch.device("cuda", torch.cuda.current_device())
    op = Operators.Float.SUM
    base = torch.randn(nkeys, dim, device=dev, generator=torch.Generator(device=dev).manual_seed(r))
    keys = [f"f{i}" for i in range(nkeys // 2)] + [f"r{r}_{i}" for i in range(nkeys - nkeys // 2)]
    m = dict(zip(keys, base.unbind(0)))
    comm.device                                                    # communicator bootstrap, untimed
    comm.barrier()
    t0 = time.perf_counter()
    out = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), op)      # first call: every key is new
    torch.cuda.synchronize()
    first_total = time.perf_counter() - t0
    assert len(out) == nkeys // 2 + p * (nkeys - nkeys // 2)
    # the agreement round alone for a dict of ALL-new keys (the key-dictionary round of a first call)
    m_new = dict(zip([f"n{r}_{i}" for i in range(nkeys)], base.unbind(0)))
    comm.barrier()
    t0 = time.perf_counter()
    assert comm._map_on_device(m_new)
    first_agree = time.perf_counter() - t0
    comm.device._keys_presynced = False
    ph = {"total": [], "walk_only": [], "agree": [], "to_tensors": [], "exchange_and_kernels": [], "to_dict": []}
    rows_list = list(m.values())
    for _ in range(iters):
        if fresh:      # a new dict object per call (same keys / rows): the full walk every call
            m = dict(zip(keys, rows_list))
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        comm.allreduceMap(m, Operands.FLOAT_OPERAND(), op)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        # the same call, phase by phase (what allreduceMap runs, in order)
        if fresh:
            m = dict(zip(keys, rows_list))
        comm.barrier()
        w0 = time.perf_counter()
        sparse._pack_native(sparse._dictionary(comm.device), m)       # the walk alone
        walk = time.perf_counter() - w0
        if fresh:
            m = dict(zip(keys, rows_list))
        comm.barrier()
        a = time.perf_counter()
        assert comm._map_on_device(m)
        b = time.perf_counter()
        eng = comm.device
        k, v, shape = sparse._map_tensors(eng, m)
        torch.cuda.synchronize()
        c = time.perf_counter()
        rk, rv = sparse.allreduce_sparse(eng, k, v, op, sparse._dictionary(eng).bits)
        torch.cuda.synchronize()
        d = time.perf_counter()
        res = sparse._tensors_map(eng, rk, rv, shape)
        e = time.perf_counter()
        assert len(res) == len(out)
        for name, dt in (("total", t1 - t0), ("walk_only", walk), ("agree", b - a), ("to_tensors", c - b),
                         ("exchange_and_kernels", d - c), ("to_dict", e - d)):
            ph[name].append(dt)
    res = {k: sorted(v)[len(v) // 2] for k, v in ph.items()}
    res["first_call_total"] = first_total
    res["first_call_agree_new_keys"] = first_agree
    return res


def main():
    from spawn_ranks import run_spawn
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--keys", type=int, default=200_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--fresh-dict", action="store_true",
                    help="a new dict object every call (no walk cache hit); default: the same dict again")
    a = ap.parse_args()
    res = run_spawn(a.p, body, args=(a.keys, a.dim, a.iters, a.fresh_dict), timeout=600)
    rec = {"config": f"allreduceMap Dict[str, float[{a.dim}]] {a.keys} keys/rank (50% shared)",
           "processes_on_one_gpu": a.p,
           "exchange_transport": ("IPC copy-plan kernels (all ranks on one GPU: not xGMI); counts over the host mesh"
                                  if os.environ.get("MP4X_SPARSE_IPC", "1") == "1" else "gloo (one GPU: not xGMI)"),
           "dict_per_call": "fresh" if a.fresh_dict else "same (walk cached by PEP 509 version tag)"}
    rec["keys_via"] = "master" if os.environ.get("MP4X_KEYS_VIA_MASTER") == "1" else "peer-to-peer host mesh"
    rec["key_hint"] = os.environ.get("MP4X_MAP_KEY_HINT", "1") == "1"
    for k in ("first_call_total", "first_call_agree_new_keys", "total", "walk_only", "agree", "to_tensors",
              "exchange_and_kernels", "to_dict"):
        rec[f"{k}_ms_max_rank"] = round(max(v[k] for v in res.values()) * 1e3, 2)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
