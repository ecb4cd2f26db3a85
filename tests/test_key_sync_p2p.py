"""Map key-dictionary rounds travel peer to peer (host mesh), not through the master.

The master keeps the placement agreement (a few bytes per rank); the new key strings go over
the data plane (``HostEngine.allgather_bytes``) — the reference's master carries control only
(J/rpc/Server.java:131-137) while map contents move slave to slave
(ProcessCommSlave.java:1329-1373)."""
import pytest

torch = pytest.importorskip("torch")

from harness import run_ranks  # noqa: E402
from mp4x.parallel.sparse import decode_keys, encode_keys  # noqa: E402


@pytest.mark.parametrize("keys", [[], ["a"], ["", "x", ""], ["ключ", "键", "k\x01"], [f"f{i}" for i in range(5000)],
                                  ["has\0nul", "b"], [1, 2, (3, "x")]])
def test_key_codec_roundtrip(keys):
    assert decode_keys(encode_keys(keys)) == keys


def test_key_codec_fast_path_is_plain_utf8():
    b = encode_keys(["ab", "c"])
    assert b == b"Sab\0c"


def _map_fn(comm, nkeys):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    before = comm.server.call("stats")
    d = {f"feature_{r}_{i}": torch.full((4,), float(i)) for i in range(nkeys)}
    d.update({f"shared_{i}": torch.full((4,), 1.0) for i in range(nkeys // 2)})
    out = comm.allreduceMap(d, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    comm.barrier()
    after = comm.server.call("stats")
    ok = len(out) == p * nkeys + nkeys // 2 and all(float(out[f"shared_{i}"][0]) == p for i in range(nkeys // 2)) \
        and all(float(out[f"feature_{j}_{i}"][1]) == i for j in range(p) for i in (0, nkeys - 1))
    return ok, after.get("allgather_obj", 0) - before.get("allgather_obj", 0)


def test_new_keys_do_not_go_through_the_master():
    nkeys = 4000          # ~60 KB of key strings per rank on the first call
    res, _, _ = run_ranks(4, _map_fn, args=(nkeys,), timeout=120)
    for r, (ok, master_bytes) in res.items():
        assert ok, r
    # every rank's control-plane bytes for the whole collective (agreement + bootstrap rounds)
    # stay far below ONE rank's key strings
    assert res[0][1] < 8000, res[0][1]
