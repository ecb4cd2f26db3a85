"""mp4x — an MI355X-native collective-communication library with the capabilities
and ``CommSlave`` API of junphine/ytk-mp4j.

Quick start (host data, any machine)::

    from mp4x import CommMaster, ProcessCommSlave, Operands, Operators
    # process 0:   CommMaster(2, 61235).start()
    comm = ProcessCommSlave("user", "127.0.0.1", 61235)
    comm.allreduceArray(arr, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, len(arr))

GPU tensors (``torch.Tensor`` on an MI355X) go through RCCL over xGMI plus the
hand-written CDNA4 HIP kernels in ``csrc/``.
"""
from .exceptions import Mp4jException, Mp4xError
from .operators import (Collective, Container, Operators, Operator, CustomOperator, OpCode, DType,
                        IDoubleOperator, IFloatOperator, ILongOperator, IIntOperator, IShortOperator,
                        IByteOperator, IStringOperator, IObjectOperator)
from .operands import Operand, Operands, Serializer, KryoUtils
from .utils.commutils import CommUtils
from .utils.scatter_allocate import ScatterAllocate
from .control.master import CommMaster
from .parallel.process_comm import ProcessCommSlave, ProcessComm
from .parallel.thread_comm import ThreadCommSlave, ThreadComm

__version__ = "0.1.0"

__all__ = [
    "Mp4jException", "Mp4xError", "Collective", "Container", "Operators", "Operator", "CustomOperator",
    "OpCode", "DType", "IDoubleOperator", "IFloatOperator", "ILongOperator", "IIntOperator",
    "IShortOperator", "IByteOperator", "IStringOperator", "IObjectOperator", "Operand", "Operands",
    "Serializer", "KryoUtils", "CommUtils", "ScatterAllocate", "CommMaster", "ProcessCommSlave",
    "ProcessComm", "ThreadCommSlave", "ThreadComm",
]
