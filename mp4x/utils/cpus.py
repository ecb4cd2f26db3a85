"""How many CPUs this process may really use.

``os.cpu_count()`` reports the machine (256 on the MI355X boxes) even when the process runs
under a cgroup CPU quota (16 CPUs there) or a narrower affinity mask; sizing host fan-outs by it
oversubscribes the quota.  The usable count is the minimum of the affinity mask, the cgroup
quota (v2 ``cpu.max`` or v1 ``cfs_quota_us / cfs_period_us``) and ``OMP_NUM_THREADS`` when set."""
from __future__ import annotations

import functools
import os


def _cgroup_quota():
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0 and per > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


@functools.lru_cache(maxsize=1)
def usable_cpus() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = _cgroup_quota()
    if q:
        n = min(n, q)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)
