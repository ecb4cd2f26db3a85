from .process_comm import ProcessCommSlave, ProcessComm

__all__ = ["ProcessCommSlave", "ProcessComm"]
