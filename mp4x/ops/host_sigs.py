"""C signatures of libmp4x_host.so (csrc/host/host_ops.cpp)."""
import ctypes

from .native import c_double, c_int, c_int64, c_void_p, PP

P64 = ctypes.POINTER(ctypes.c_int64)

HOST_SIGS = {
    "mp4x_host_reduce": (c_int, [c_int, c_int, c_void_p, PP, c_int, c_int64, c_int]),
    "mp4x_host_threads": (c_int, []),
    "mp4x_shm_header_bytes": (c_int64, []),
    "mp4x_shm_attach": (c_void_p, [c_void_p, c_int, c_int, c_int64, c_int, c_double]),
    "mp4x_shm_detach": (None, [c_void_p]),
    "mp4x_shm_barrier": (c_int, [c_void_p]),
    "mp4x_shm_watch_peers": (c_int, [c_void_p]),
    "mp4x_shm_allreduce": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int64]),
    "mp4x_shm_reduce_scatter": (c_int, [c_void_p, c_int, c_int, c_void_p, P64, P64]),
    "mp4x_shm_allgather": (c_int, [c_void_p, c_int, c_void_p, P64, P64]),
    "mp4x_shm_broadcast": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_int]),
    "mp4x_tbarrier_create": (c_void_p, [c_int, c_double]),
    "mp4x_tbarrier_destroy": (None, [c_void_p]),
    "mp4x_tbarrier_abort": (None, [c_void_p]),
    "mp4x_tbarrier_aborted": (c_int, [c_void_p]),
    "mp4x_tbarrier_wait": (c_int, [c_void_p]),
    "mp4x_team_create": (c_void_p, [c_int, c_double]),
    "mp4x_team_destroy": (None, [c_void_p]),
    "mp4x_team_abort": (None, [c_void_p]),
    "mp4x_team_barrier": (c_int, [c_void_p, c_int]),
    "mp4x_team_aborted": (c_int, [c_void_p]),
    "mp4x_team_reduce": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_int, c_int, c_int]),
    "mp4x_team_bcast": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_int, c_int]),
    "mp4x_team_allreduce": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_int, c_int]),
}
