"""CommUtils / ScatterAllocate semantics (reference J/utils/CommUtils.java, J/utils/ScatterAllocate.java)."""
import pytest

from mp4x import CommUtils, Mp4jException
from mp4x.utils.scatter_allocate import plan, recv_num, allocate
from mp4x.utils.hashing import java_string_hash, owner_of


def test_process_partitions_match_reference_main():
    # CommUtils.main prints these for size=101, slaveNum=4 (CommUtils.java:224-238)
    assert CommUtils.createProcessArrayFroms(101, 4) == [0, 25, 50, 75]
    assert CommUtils.createProcessArrayTos(101, 4) == [25, 50, 75, 101]
    f = CommUtils.createThreadArrayFroms(101, 4, 2)
    t = CommUtils.createThreadArrayTos(101, 4, 2)
    assert f == [[0, 12], [25, 37], [50, 62], [75, 88]]
    assert t == [[12, 25], [37, 50], [62, 75], [88, 101]]


def test_counts_to_ranges():
    assert CommUtils.getFromsFromCount(5, [2, 0, 3], 3) == [5, 7, 7]
    assert CommUtils.getTosFromCount(5, [2, 0, 3], 3) == [7, 7, 10]
    assert CommUtils.even_split(10, 21, 3) == ([10, 13, 16], [13, 16, 21], [3, 3, 5])


@pytest.mark.parametrize("froms,tos", [([0, 5], [5]), ([-1], [3]), ([0], [-2]), ([4], [3]), ([0, 2], [3, 4])])
def test_illegal_ranges_raise(froms, tos):
    with pytest.raises(Mp4jException):
        CommUtils.isfromsTosLegal(froms, tos)


def test_legal_ranges_and_2d():
    CommUtils.isfromsTosLegal([0, 3, 3], [3, 3, 9])
    f = CommUtils.createThreadArrayFroms(100, 3, 4)
    t = CommUtils.createThreadArrayTos(100, 3, 4)
    CommUtils.isfromsTosLegal2D(f, t, 4)
    with pytest.raises(Mp4jException):
        CommUtils.isfromsTosLegal2D(f, t, 3)
    with pytest.raises(Mp4jException):
        CommUtils.isFromToLegal(5, 4)
    with pytest.raises(Mp4jException):
        CommUtils.isFromCountsLegal(0, [1, -1])
    with pytest.raises(Mp4jException):
        CommUtils.isFromCountsLegal(0, [[1], [-1]])


def test_scatter_plan_examples_from_survey():
    # SURVEY Appendix A.3 (simulated from ScatterAllocate.allocate)
    assert allocate(8, 0) == {0: [(0, 4, 4, 7), (0, 2, 2, 3), (0, 1, 1, 1)], 2: [(2, 3, 3, 3)],
                              4: [(4, 6, 6, 7), (4, 5, 5, 5)], 6: [(6, 7, 7, 7)]}
    assert allocate(8, 3)[3] == [(3, 0, 0, 3), (3, 4, 4, 7)]
    assert allocate(6, 0) == {0: [(0, 3, 3, 5), (0, 1, 1, 2)], 1: [(1, 2, 2, 2)], 3: [(3, 4, 4, 5)],
                              4: [(4, 5, 5, 5)]}
    assert allocate(3, 1) == {1: [(1, 0, 0, 0), (1, 2, 2, 2)]}


@pytest.mark.parametrize("p", list(range(2, 40)))
def test_scatter_plan_every_rank_receives_at_most_once(p):
    # the reference self-test ScatterAllocate.main (:36-56) for p = 13, here for 2..39
    for root in range(p):
        cnt = recv_num(p, root)
        assert all(v <= 1 for v in cnt.values())
        assert all(cnt.get(r, 0) == 1 for r in range(p) if r != root)


def test_java_string_hash():
    # values of java.lang.String.hashCode
    assert java_string_hash("") == 0
    assert java_string_hash("a") == 97
    assert java_string_hash("hello") == 99162322
    assert java_string_hash("polygenelubricants") == -2147483648
    assert java_string_hash("-1") == 1444
    assert owner_of("polygenelubricants", 3) == (-(2147483648 % 3)) % 3
