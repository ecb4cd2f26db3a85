"""Dense, rank-consistent map-key ids (parallel/sparse.py KeyDictionary): every rank numbers a
sync round's union in the same order, ids stay dense, and ``bits`` bounds the sort width."""
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
