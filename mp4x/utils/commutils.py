"""Range validation and block partitioning.

Same semantics (and error conditions) as the reference's ``CommUtils``
(/root/reference/src/main/java/com/fenbi/mp4j/utils/CommUtils.java:34-222):
ranges are half-open ``[from, to)``, partitions give every part
``size // parts`` elements and the LAST part the remainder.  Indices are Python
ints (int64 semantics on the device side) instead of Java's 31-bit ``int``.
"""
from __future__ import annotations

from typing import List, Sequence

from ..exceptions import RangeError


class CommUtils:
    # ---------------------------------------------------------------- validation
    @staticmethod
    def isfromsTosLegal(froms: Sequence[int], tos: Sequence[int]) -> None:
        """1-D check (CommUtils.java:34-58)."""
        if len(froms) != len(tos):
            raise RangeError("froms, tos's length must be equal!")
        for i in range(len(froms)):
            if froms[i] < 0:
                raise RangeError("froms[i] must be >= 0!")
            if tos[i] < 0:
                raise RangeError("tos[i] must be >= 0!")
            if froms[i] > tos[i]:
                raise RangeError("froms[i] must be <= tos[i]!")
            if i >= 1 and froms[i] < tos[i - 1]:
                raise RangeError("froms[i] must be >= to[i - 1]")

    @staticmethod
    def isfromsTosLegal2D(froms: Sequence[Sequence[int]], tos: Sequence[Sequence[int]], threadNum: int) -> None:
        """2-D ``[slave][thread]`` check (CommUtils.java:60-81)."""
        for i in range(len(froms)):
            CommUtils.isfromsTosLegal(froms[i], tos[i])
            if len(froms[i]) != threadNum:
                raise RangeError("froms arrays must be array[slaveNum][threadNum]")
            if len(tos[i]) != threadNum:
                raise RangeError("tos arrays must be array[slaveNum][threadNum]")
        CommUtils.isfromsTosLegal(CommUtils.getProcessFroms(froms), CommUtils.getProcessTos(tos))

    @staticmethod
    def isFromCountsLegal(frm: int, counts) -> None:
        """1-D or 2-D counts check (CommUtils.java:83-107)."""
        if frm < 0:
            raise RangeError("from must be >= 0!")
        for c in counts:
            if isinstance(c, (list, tuple)):
                for cc in c:
                    if cc < 0:
                        raise RangeError("counts[i][j] must be >= 0!")
            elif c < 0:
                raise RangeError("counts[i] must be >= 0!")

    @staticmethod
    def isFromToLegal(frm: int, to: int) -> None:
        """CommUtils.java:128-140."""
        if frm < 0:
            raise RangeError("from must be >= 0!")
        if to < 0:
            raise RangeError("to must be >= 0!")
        if frm > to:
            raise RangeError("from must be <= to!")

    # ---------------------------------------------------------------- conversion
    @staticmethod
    def getFromsFromCount(frm: int, counts: Sequence[int], slaveNum: int) -> List[int]:
        out = []
        for i in range(slaveNum):
            out.append(frm)
            frm += counts[i]
        return out

    @staticmethod
    def getTosFromCount(frm: int, counts: Sequence[int], slaveNum: int) -> List[int]:
        out = []
        for i in range(slaveNum):
            frm += counts[i]
            out.append(frm)
        return out

    @staticmethod
    def getProcessFroms(froms: Sequence[Sequence[int]]) -> List[int]:
        return [row[0] for row in froms]

    @staticmethod
    def getProcessTos(tos: Sequence[Sequence[int]]) -> List[int]:
        return [row[-1] for row in tos]

    # ---------------------------------------------------------------- partitions
    @staticmethod
    def createProcessArrayFroms(size: int, slaveNum: int) -> List[int]:
        avg = size // slaveNum
        return [r * avg for r in range(slaveNum)]

    @staticmethod
    def createProcessArrayTos(size: int, slaveNum: int) -> List[int]:
        avg = size // slaveNum
        tos = [(r + 1) * avg for r in range(slaveNum)]
        tos[-1] = size
        return tos

    @staticmethod
    def createThreadArrayFroms(size: int, slaveNum: int, threadNum: int) -> List[List[int]]:
        pf = CommUtils.createProcessArrayFroms(size, slaveNum)
        pt = CommUtils.createProcessArrayTos(size, slaveNum)
        return [[f + pf[r] for f in CommUtils.createProcessArrayFroms(pt[r] - pf[r], threadNum)]
                for r in range(slaveNum)]

    @staticmethod
    def createThreadArrayTos(size: int, slaveNum: int, threadNum: int) -> List[List[int]]:
        pf = CommUtils.createProcessArrayFroms(size, slaveNum)
        pt = CommUtils.createProcessArrayTos(size, slaveNum)
        return [[t + pf[r] for t in CommUtils.createProcessArrayTos(pt[r] - pf[r], threadNum)]
                for r in range(slaveNum)]

    # ---------------------------------------------------------------- helpers used by the engines
    @staticmethod
    def even_split(frm: int, to: int, parts: int):
        """``[from,to)`` into ``parts`` blocks, last takes the remainder.

        This is the split used by allreduce / reduce / broadcast
        (ProcessCommSlave.java:1741-1756, :750-760, :1397-1412).
        Returns ``(froms, tos, counts)``.
        """
        avg = (to - frm) // parts
        froms = [frm + r * avg for r in range(parts)]
        tos = [f + avg for f in froms]
        tos[-1] = to
        counts = [t - f for f, t in zip(froms, tos)]
        return froms, tos, counts
