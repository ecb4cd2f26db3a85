"""Binary-tree scatter / gather plans.

Same plan as the reference's ``ScatterAllocate.allocate``
(/root/reference/src/main/java/com/fenbi/mp4j/utils/ScatterAllocate.java:58-111):
the root hands ``[0, mid)`` to rank 0 and ``[mid, p)`` to rank ``mid`` (skipping a
hand-off to itself), then every range is recursively halved.  A task
``(src, dst, rank_from, rank_to)`` means "src sends the segments owned by ranks
``rank_from..rank_to`` (inclusive) to dst".  Every non-root rank is the ``dst``
of exactly one task (checked by :func:`recv_num`, the reference's self-test
``ScatterAllocate.main`` :36-56).

The same plan reversed is the deterministic gather tree used by
``gatherArray``/``gatherMap`` (the reference pairs ranks dynamically through
the master's ``Exchanger``; a fixed binomial tree needs no master round-trips).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Tuple

Task = Tuple[int, int, int, int]


def _split(start: int, end: int, out: List[Task]) -> None:
    # iterative version of ScatterAllocate.split (:97-111), same emission order
    stack = [(start, end)]
    while stack:
        s, e = stack.pop()
        if s >= e:
            continue
        half = (e - s + 1) // 2
        out.append((s, s + half, s + half, e))
        # recursion order: left half first, then right half
        stack.append((s + half, e))
        stack.append((s, s + half - 1))


def plan(p: int, root: int) -> List[Task]:
    """Ordered task list for p ranks rooted at ``root``."""
    if p <= 1:
        return []
    mid = p // 2
    tasks: List[Task] = []
    if root != 0:
        tasks.append((root, 0, 0, mid - 1))
    if root != mid:
        tasks.append((root, mid, mid, p - 1))
    _split(0, mid - 1, tasks)
    _split(mid, p - 1, tasks)
    return tasks


def allocate(p: int, root: int) -> Dict[int, List[Task]]:
    """Reference-shaped result: ``src -> [tasks]`` in emission order."""
    m: Dict[int, List[Task]] = defaultdict(list)
    for t in plan(p, root):
        m[t[0]].append(t)
    return dict(m)


def recv_num(p: int, root: int) -> Dict[int, int]:
    cnt: Dict[int, int] = defaultdict(int)
    for t in plan(p, root):
        cnt[t[1]] += 1
    return dict(cnt)


class ScatterAllocate:
    """Namespace with the reference's method names."""
    allocate = staticmethod(allocate)
    recvNum = staticmethod(recv_num)
    plan = staticmethod(plan)
