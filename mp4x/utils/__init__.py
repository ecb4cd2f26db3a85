from .commutils import CommUtils
from .scatter_allocate import ScatterAllocate
from .hashing import java_string_hash, owner_of, key_id, key_ids

__all__ = ["CommUtils", "ScatterAllocate", "java_string_hash", "owner_of", "key_id", "key_ids"]
