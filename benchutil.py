"""Host facts the benchmarks report beside their CPU baselines (not product code).

`host_cores()` answers "how many host cores does this process really have": the CPUs in its affinity mask
(what `nproc` shows; on a GPU box that is the whole machine) and the CPU quota of its cgroup (the box's
share of them, e.g. 16 per GPU).  The CPU baselines run on `usable` = the smaller of the two and report
both, so the core count of a baseline is the box's, not a fixed cap (host hardware
concurrency).
"""
from __future__ import annotations

import os


def _cgroup_quota_cores():
    """CPU quota of this process's cgroup in cores (cgroup v2 `cpu.max`, else v1 cfs files), or None."""
    try:
        with open("/proc/self/cgroup") as f:
            lines = f.read().splitlines()
    except OSError:
        lines = []
    paths = []
    for ln in lines:
        parts = ln.split(":", 2)
        if len(parts) == 3 and (parts[0] == "0" or "cpu" in parts[1].split(",")):
            paths.append(parts[2])
    for rel in paths + ["/"]:
        for base in ("/sys/fs/cgroup", "/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
            d = os.path.join(base, rel.lstrip("/"))
            try:
                with open(os.path.join(d, "cpu.max")) as f:
                    q, p = f.read().split()[:2]
                if q != "max" and int(p) > 0:
                    return max(1, int(q) // int(p))
            except (OSError, ValueError):
                pass
            try:
                with open(os.path.join(d, "cpu.cfs_quota_us")) as f:
                    q = int(f.read())
                with open(os.path.join(d, "cpu.cfs_period_us")) as f:
                    p = int(f.read())
                if q > 0 and p > 0:
                    return max(1, q // p)
            except (OSError, ValueError):
                pass
    return None


def host_cores() -> dict:
    """{"affinity": CPUs in the affinity mask, "cgroup_quota": the cgroup's CPU quota in cores (None = no
    quota), "omp_share": OMP_NUM_THREADS as the box advertises its CPU share (None = unset), "usable": the
    smallest of them}."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = _cgroup_quota_cores()
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "")) or None
    except ValueError:
        share = None
    usable = min(x for x in (aff, quota, share) if x)
    return {"affinity": aff, "cgroup_quota": quota, "omp_share": share, "usable": max(1, usable)}
