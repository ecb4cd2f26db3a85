from .master import CommMaster
from .client import MasterClient

__all__ = ["CommMaster", "MasterClient"]
