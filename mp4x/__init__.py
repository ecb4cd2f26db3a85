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
import os as _os
import sys as _sys

# Cross-process device memory (hipIpc handles, RCCL's peer buffers) goes through dmabuf on this
# platform; the legacy IPC mode fails there with "hipIpcGetMemHandle: invalid argument".  Read by
# the HSA runtime at its first use, so it only takes effect when mp4x is imported before anything
# touches the GPU; an explicit setting is kept.  What was in effect is recorded (IPC_MODE_AT_IMPORT)
# so a failing handle export can name the cause (mp4x.parallel.ipc.ipc_mode_report).
_t = _sys.modules.get("torch")
try:
    _hip_up = bool(_t is not None and _t.cuda.is_initialized())
except Exception:   # noqa: BLE001 — a partially imported torch
    _hip_up = False
IPC_MODE_AT_IMPORT = {"env_before_import": _os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"),
                      "hip_initialized_before_import": _hip_up}
del _t, _hip_up
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from .exceptions import Mp4jException, Mp4xError  # noqa: E402
from .operators import (Collective, Container, Operators, Operator, CustomOperator, OpCode, DType,  # noqa: E402
                        IDoubleOperator, IFloatOperator, ILongOperator, IIntOperator, IShortOperator,
                        IByteOperator, IStringOperator, IObjectOperator)
from .operands import Operand, Operands, Serializer, KryoUtils  # noqa: E402
from .utils.commutils import CommUtils  # noqa: E402
from .utils.scatter_allocate import ScatterAllocate  # noqa: E402
from .control.master import CommMaster  # noqa: E402
from .parallel.process_comm import ProcessCommSlave, ProcessComm  # noqa: E402
from .parallel.thread_comm import ThreadCommSlave, ThreadComm  # noqa: E402

__version__ = "0.1.0"

__all__ = [
    "Mp4jException", "Mp4xError", "Collective", "Container", "Operators", "Operator", "CustomOperator",
    "OpCode", "DType", "IDoubleOperator", "IFloatOperator", "ILongOperator", "IIntOperator",
    "IShortOperator", "IByteOperator", "IStringOperator", "IObjectOperator", "Operand", "Operands",
    "Serializer", "KryoUtils", "CommUtils", "ScatterAllocate", "CommMaster", "ProcessCommSlave",
    "ProcessComm", "ThreadCommSlave", "ThreadComm",
]
