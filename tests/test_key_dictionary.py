"""Dense, rank-consistent map-key ids (parallel/sparse.py KeyDictionary): every rank numbers a
sync round's union in the same order, ids stay dense, and ``bits`` bounds the sort width."""
import pytest

from mp4x.parallel.sparse import KeyDictionary


def test_rounds_number_the_union_identically_on_every_rank():
    proposals = [["b", "a", "b"], [], ["a", "c"], ["d"]]       # what p = 4 ranks saw first
    ds = [KeyDictionary() for _ in range(4)]
    for r, d in enumerate(ds):
        assert d.unknown(proposals[r]) == list(dict.fromkeys(proposals[r]))
        d.learn_round([list(dict.fromkeys(x)) for x in proposals])
    assert all(d.id2key == ["b", "a", "c", "d"] for d in ds)
    assert ds[0].ids(["d", "a"]) == [3, 1]
    # second round: only unseen keys travel; ids continue densely
    for d in ds:
        assert d.unknown(["a", "e", "f", "e"]) == ["e", "f"]
        d.learn_round([["e", "f"], ["f", "g"], [], []])
    assert ds[2].ids(["e", "f", "g"]) == [4, 5, 6]
    assert ds[1].bits == 3                     # ids 0..6


def test_bits_small_dictionaries():
    d = KeyDictionary()
    assert d.bits == 1
    d.learn_round([[1]])
    assert d.bits == 1
    d.learn_round([[2, 3]])
    assert d.bits == 2                          # ids 0..2
    d.learn_round([list(range(100, 1100))])
    assert d.bits == (len(d.id2key) - 1).bit_length()


def test_tensor_map_is_a_dict_view():
    """The device map collectives return a lazy mapping over (ids, rows): dict semantics,
    mutation through an overlay, and the unmodified map goes back in without per-key work."""
    import numpy as np
    import torch
    from mp4x.parallel.sparse import KeyDictionary, TensorMap, _map_tensors

    d = KeyDictionary()
    d.learn_round([["a", "b", "c"]])
    rows = torch.arange(12, dtype=torch.float32).view(3, 4)
    m = TensorMap(d, np.array([2, 0, 1], dtype=np.int64), rows, (2, 2))
    assert list(m) == ["c", "a", "b"] and len(m) == 3
    assert torch.equal(m["a"], rows[1].view(2, 2)) and "b" in m and "z" not in m
    assert dict(m.items()).keys() == {"a", "b", "c"}

    class _Eng:
        _keydict = d
        device = torch.device("cpu")
        _keys_presynced = True              # the collective key round is skipped in this unit test
    ids, v, shape = _map_tensors(_Eng, m)
    assert ids.tolist() == [2, 0, 1] and v.data_ptr() == rows.data_ptr() and shape == (2, 2)

    m["z"] = torch.zeros(2, 2)
    del m["a"]
    assert list(m) == ["c", "b", "z"] and len(m) == 3 and "a" not in m
    m["a"] = torch.ones(2, 2)
    assert len(m) == 4 and torch.equal(m["a"], torch.ones(2, 2))
    del m["z"]
    assert len(m) == 3 and not m.pristine()


def test_rows_of_one_base_detection():
    """The dict->rows fast path (sparse._rows_of_one_base) accepts only whole rows of one
    contiguous base; everything else goes through torch.stack."""
    import random

    import torch
    from mp4x.parallel.sparse import _rows_of_one_base
    base = torch.randn(3000, 16)
    vals = list(base.unbind(0))
    perm = list(range(3000))
    random.Random(0).shuffle(perm)
    sub = [vals[i] for i in perm[:2000]]
    idx = _rows_of_one_base(sub)
    assert idx is not None and torch.equal(base.index_select(0, idx), torch.stack(sub))
    sq = torch.randn(64, 64)
    assert _rows_of_one_base([sq[:, i] for i in range(64)]) is None          # columns
    assert _rows_of_one_base([sq[i, :32] for i in range(64)]) is None        # half rows
    assert _rows_of_one_base(vals[:10] + list(torch.randn(4, 16).unbind(0))) is None   # two bases
    t = torch.randn(500, 8)
    rows = list(t[100:400].unbind(0))                                         # rows of a slice
    assert torch.equal(t.index_select(0, _rows_of_one_base(rows)), torch.stack(rows))
    t3 = torch.randn(50, 4, 8)
    idx3 = _rows_of_one_base(list(t3.unbind(0)))                              # [4, 8] slabs
    assert torch.equal(idx3, torch.arange(50))


def test_lookup_marks_unseen_keys():
    d = KeyDictionary()
    d.learn_round([["a", "b"]])
    assert d.lookup(["b", "x", "a", "x"]).tolist() == [1, -1, 0, -1]


def _python_form(d, m):
    """What the Python path computes: ids (-1 when unknown) and the stacked rows."""
    import numpy as np
    import torch
    ids = d.lookup(list(m.keys()))
    rows = torch.stack([v.reshape(-1) for v in m.values()])
    return ids, rows


def test_native_map_pack_matches_the_python_form():
    """csrc/pyext/map_ext.cpp: one dict walk gives the same ids as ``KeyDictionary.lookup`` and
    rows only when EVERY value is a whole contiguous row of the first value's base tensor of the
    same dtype; anything else falls back to one stack with identical values."""
    import numpy as np
    import pytest
    import torch
    from mp4x.ops import native
    from mp4x.parallel import sparse

    if native.map_ext() is None:
        pytest.skip("_mp4x_map not built")
    base = torch.arange(40 * 6, dtype=torch.float32).view(40, 6)
    d = KeyDictionary()
    d.learn_round([[f"k{i}" for i in range(0, 40, 2)]])
    cases = {
        "rows in order": {f"k{i}": base[i] for i in range(40)},
        "rows shuffled": {f"k{i}": base[i] for i in (5, 3, 39, 0, 17)},
        "foreign value": {**{f"k{i}": base[i] for i in range(4)}, "x": torch.zeros(6)},
        "other dtype view": {"k0": base[0], "k1": base[1].view(torch.int32)},
        "partial rows": {"k0": base[0, :3], "k2": base[2, 3:]},     # rows of base as [80, 3]
        "misaligned": {"k0": base[0, :3], "k2": base[2, 1:4]},
        "strided row": {"k0": base[:, 0], "k2": base[:, 1]},
        "2-D values": {f"k{i}": base.view(20, 2, 6)[i] for i in range(20)},
    }
    expect_rows = {"rows in order": True, "rows shuffled": True, "2-D values": True, "partial rows": True}
    for name, m in cases.items():
        ids, nmiss, rows, b = sparse._pack_native(d, m)
        ref_ids, ref_rows = _python_form(d, m)
        assert np.array_equal(ids, ref_ids), name
        assert nmiss == int((ref_ids < 0).sum()), name
        assert (rows is not None) == expect_rows.get(name, False), name
        if rows is not None:
            got = b.reshape(-1, ref_rows.shape[1]).index_select(0, torch.from_numpy(rows))
            assert torch.equal(got, ref_rows), name
    # non-dict mappings and empty maps take the Python path
    from collections import OrderedDict
    assert sparse._pack_native(d, OrderedDict(k0=base[0])) is None
    assert sparse._pack_native(d, {}) is None
    assert sparse._pack_native(d, {"k0": [1.0, 2.0]}) is None


def test_native_host_partition_matches_java_hash_rule():
    """csrc/pyext/hostmap_ext.cpp ``partition``: owner = Java String.hashCode % p (signed
    remainder, negatives wrapped) exactly as utils/hashing.owner_of, incl. non-BMP keys (UTF-16
    surrogate pairs), insertion order kept per part; non-str keys defer to Python."""
    import random

    import pytest
    from mp4x.ops import native
    from mp4x.utils.hashing import owner_of

    ext = native.hostmap_ext()
    if ext is None:
        pytest.skip("_mp4x_hostmap not built")
    rng = random.Random(7)
    keys = ["", "a", "hello", "f123", "é", "日本語", "😀x", "\U0010ffff", "a" * 100]
    for _ in range(2000):
        keys.append("".join(chr(rng.choice([rng.randint(32, 126), rng.randint(160, 0xD7FF),
                                            rng.randint(0x10000, 0x10FFFF)])) for _ in range(rng.randint(0, 12))))
    m = {k: i for i, k in enumerate(keys)}
    for p in (1, 2, 3, 5, 7, 8):
        parts = ext.partition(m, p)
        assert sum(map(len, parts)) == len(m)
        for r, d in enumerate(parts):
            assert all(owner_of(k, p) == r for k in d)
            assert list(d) == [k for k in m if owner_of(k, p) == r]       # insertion order
    assert ext.partition({1: 2}, 2) is None


def test_native_stack_rows_and_vectorised_merge():
    """``wire.stack_rows`` / ``merge_reduce`` with numpy rows equal the per-key reference."""
    import numpy as np
    from mp4x import Operators
    from mp4x.parallel import wire

    rng = np.random.default_rng(0)
    rows = [rng.standard_normal(5).astype(np.float32) for _ in range(50)]
    assert np.array_equal(wire.stack_rows(rows), np.stack(rows))
    assert np.array_equal(wire.stack_rows(rows, np.float64), np.stack(rows).astype(np.float64))
    mixed = rows[:3] + [rows[3].astype(np.float64)]
    assert np.array_equal(wire.stack_rows(mixed), np.stack(mixed))            # falls back
    local = {f"k{i}": rows[i].copy() for i in range(0, 50, 2)}
    keys = [f"k{i}" for i in range(50)]
    vals = np.stack(rows[::-1])
    for op in (Operators.Float.SUM, Operators.Float.MAX):
        expect = {k: v.copy() for k, v in local.items()}
        for k, row in zip(keys, vals):
            if k in expect:
                op.reduce_into(expect[k], row)
            else:
                expect[k] = row
        got = wire.merge_reduce({k: v.copy() for k, v in local.items()}, keys, vals, op)
        assert got.keys() == expect.keys()
        assert all(np.array_equal(got[k], expect[k]) for k in keys)
    # a shared local value of another dtype takes the per-key path (its dtype is kept)
    odd = {"k0": rows[0].astype(np.float64)}
    got = wire.merge_reduce(odd, keys[:2], vals[:2], Operators.Float.SUM)
    assert got["k0"].dtype == np.float64 and np.allclose(got["k0"], rows[0] + vals[0])


def test_native_partition_property():
    """Hypothesis: any str keys (any code points, incl. lone surrogates, which Java also hashes
    as code units), any p: the native partition equals the Python rule."""
    import pytest
    hyp = pytest.importorskip("hypothesis")
    st = hyp.strategies
    from mp4x.ops import native
    from mp4x.utils.hashing import owner_of

    ext = native.hostmap_ext()
    if ext is None:
        pytest.skip("_mp4x_hostmap not built")

    def java_units(s):           # owner_of via UTF-16 code units (surrogatepass for lone ones)
        h = 0
        b = s.encode("utf-16-be", "surrogatepass")
        for i in range(0, len(b), 2):
            h = (31 * h + ((b[i] << 8) | b[i + 1])) & 0xFFFFFFFF
        return h - (1 << 32) if h >= (1 << 31) else h

    @hyp.settings(max_examples=200, deadline=None)
    @hyp.given(st.lists(st.text(max_size=20), max_size=60, unique=True), st.integers(1, 9))
    def check(keys, p):
        parts = ext.partition({k: None for k in keys}, p)
        if not keys:
            assert parts == [{} for _ in range(p)]
            return
        for r, d in enumerate(parts):
            for k in d:
                h = java_units(k)
                idx = abs(h) % p
                if h < 0 and idx:
                    idx = p - idx
                assert idx == r
                if not any(0xD800 <= ord(c) <= 0xDFFF for c in k):
                    assert owner_of(k, p) == r
        assert sum(map(len, parts)) == len(keys)
    check()


def test_tensor_map_with_tensor_ids_is_lazy():
    """A TensorMap made from an id TENSOR (what the device collectives return) converts the ids
    to the host only on first key access, and hands the same id tensor back when fed into the
    next map collective unmodified."""
    import torch
    from mp4x.parallel.sparse import KeyDictionary, TensorMap, _map_tensors

    d = KeyDictionary()
    d.learn_round([["a", "b", "c"]])
    ids = torch.tensor([2, 0], dtype=torch.int64)
    rows = torch.arange(8.0).view(2, 4)
    tm = TensorMap(d, ids, rows, (4,))
    assert len(tm) == 2 and tm._ids_np is None            # nothing converted yet

    class Eng:                                             # no sync round needed: pristine map
        _keydict = d
        device = torch.device("cpu")
        _keys_presynced = True
    k, v, shape = _map_tensors(Eng, tm)
    assert k is ids and torch.equal(v, rows) and shape == (4,) and tm._ids_np is None
    assert list(tm) == ["c", "a"] and torch.equal(tm["a"], rows[1])
    assert tm._ids_np is not None


def test_walk_cache_follows_the_dict_version():
    """The device Map API skips the dict walk for the same dict passed again unmodified (equal
    PEP 509 version tag) and walks again after any insert / delete / value replacement."""
    import numpy as np
    import pytest
    import torch
    from mp4x.ops import native
    from mp4x.parallel import sparse

    if native.map_ext() is None:
        pytest.skip("_mp4x_map not built")
    base = torch.arange(24.0).view(6, 4)
    d = KeyDictionary()
    d.learn_round([[f"k{i}" for i in range(7)]])
    m = {f"k{i}": base[i] for i in range(6)}
    ids1, n1, rows1, _ = sparse._pack_native(d, m)
    assert d._walk_cache is not None and d._walk_cache[1] is m
    ids2, n2, rows2, _ = sparse._pack_native(d, m)            # cache hit: equal results, own copies
    assert np.array_equal(ids1, ids2) and np.array_equal(rows1, rows2) and ids2 is not d._walk_cache[3]
    m["k1"] = base[5]                                         # value replaced -> new version
    ids3, _, rows3, _ = sparse._pack_native(d, m)
    assert rows3[1] == 5
    m["k6"] = torch.zeros(4)                                  # foreign value -> no rows
    ids4, _, rows4, _ = sparse._pack_native(d, m)
    assert rows4 is None and ids4[-1] == 6
    m2 = {"k0": base[0], "new": base[1]}                      # a miss is never cached
    _, nm, _, _ = sparse._pack_native(d, m2)
    assert nm == 1 and d._walk_cache is None


def test_native_learn_round_matches_python_union():
    """csrc/pyext/hostmap_ext.cpp ``learn_keys`` numbers exactly what the Python union does:
    rank order, first occurrence, known keys skipped, None blocks, any hashable key."""
    from mp4x.ops import native
    from mp4x.parallel.sparse import KeyDictionary
    ext = native.hostmap_ext()
    if ext is None:
        pytest.skip("native host-map extension not built")
    props = [["a", "b", ("t", 1), "a"], None, [], ["c", "b", 7, "known"], ["d", ("t", 1)]]
    nat = KeyDictionary()
    nat.key2id, nat.id2key = {"known": 0}, ["known"]
    assert ext.learn_keys(nat.key2id, nat.id2key, props) == 6
    ref = KeyDictionary()
    ref.key2id, ref.id2key = {"known": 0}, ["known"]
    import itertools
    union = dict.fromkeys(itertools.chain.from_iterable(b for b in props if b))
    new = [k for k in union if k not in ref.key2id]
    ref.key2id.update(zip(new, range(1, 1 + len(new))))
    ref.id2key.extend(new)
    assert nat.key2id == ref.key2id and nat.id2key == ref.id2key
    assert nat.id2key == ["known", "a", "b", ("t", 1), "c", 7, "d"]
    with pytest.raises(TypeError):
        ext.learn_keys({}, [], [[["unhashable"]]])


def test_native_walk_position_hint():
    """The native walk's position hint (same key objects, same order as the last complete walk):
    pointer compares replace dictionary probes; any other key — a new object with an equal value,
    a moved key, an unknown key — still takes the probe, so ids are always those of key2id."""
    import numpy as np
    import torch
    from mp4x.ops import native
    from mp4x.parallel.sparse import KeyDictionary, _pack_native
    ext = native.map_ext()
    if ext is None:
        pytest.skip("_mp4x_map not built")
    d = KeyDictionary()
    keys = [f"k{i}" for i in range(1000)]
    d.learn_round([keys])
    base = torch.randn(1000, 4)
    rows = base.unbind(0)

    def walk(ks, vals):
        return _pack_native(d, dict(zip(ks, vals)))

    ids, nmiss, rr, _ = walk(keys, rows)
    assert nmiss == 0 and np.array_equal(ids, np.arange(1000)) and np.array_equal(rr, np.arange(1000))
    assert d._hint is not None and len(d._hint[0]) == 1000
    m = dict(zip(keys, rows))
    out = np.empty(1000, dtype=np.int64)
    r2 = np.empty(1000, dtype=np.int64)
    _, _, hits, _ = ext.pack(m, d.key2id, base, out, r2, d._hint[0], d._hint[1], False)
    assert hits == 1000 and np.array_equal(out, np.arange(1000))
    # equal-valued new objects, a reversed order, and a key the dictionary has never seen
    fresh = ["%s" % k for k in keys[:10]] + keys[10:]
    ids, nmiss, _, _ = walk(fresh, rows)
    assert nmiss == 0 and np.array_equal(ids, np.arange(1000))
    ids, nmiss, _, _ = walk(list(reversed(keys)), rows)
    assert nmiss == 0 and np.array_equal(ids, np.arange(999, -1, -1))
    ids, nmiss, _, _ = walk(keys[:500] + ["new"] + keys[501:], rows)
    assert nmiss == 1 and ids[500] == -1 and np.array_equal(np.delete(ids, 500), np.delete(np.arange(1000), 500))
    # a walk with a miss keeps the previous hint
    assert len(d._hint[0]) == 1000 and d._hint[0][0] == "k999"
