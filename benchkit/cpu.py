"""Host CPU facts for the bench line: where a thread ran (CPU, clock, NUMA
node), the speculation state that moves the CPU baseline 19x between boxes
(DESIGN.md §5 Host variance), the CPU quota, and each rank's pinning to its
GPU's NUMA node."""
from __future__ import annotations

import contextlib
import os

from storb_amd import _lib


def cpu_where(cpu):
    """Clock and NUMA node of logical CPU `cpu` (from /proc and /sys)."""
    mhz, node = None, None
    try:
        cur = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("processor"):
                cur = int(line.split(":")[1])
            elif line.startswith("cpu MHz") and cur == cpu:
                mhz = float(line.split(":")[1])
                break
    except (OSError, ValueError):
        pass
    try:
        for name in os.listdir(f"/sys/devices/system/cpu/cpu{cpu}"):
            if name.startswith("node") and name[4:].isdigit():
                node = int(name[4:])
    except OSError:
        pass
    return {"cpu": cpu, "cpu_mhz": mhz, "numa_node": node}


def ssbd_run(run, secs):
    """run(fresh=True, secs) on a fresh thread that first turns SSBD on for
    itself (PR_SET_SPECULATION_CTRL; irreversible for that thread only)."""
    import ctypes
    import threading
    res = {}

    def body():
        libc = ctypes.CDLL(None, use_errno=True)
        rc = libc.prctl(53, 0, 4, 0, 0)  # PR_SET_SPECULATION_CTRL, PR_SPEC_STORE_BYPASS, DISABLE
        if rc != 0:
            res["refused_errno"] = ctypes.get_errno()
            return
        v, c, e, a = run(True, secs)
        res.update({"value": v, "unit": "GiB/s", "calls": c, "seconds": round(e, 2),
                    "ipc": a.get("ipc"), "effective_ghz": a.get("effective_ghz"),
                    "l1_addmul_GBps": a.get("l1_addmul_GBps"),
                    "Speculation_Store_Bypass": a["speculation"].get("Speculation_Store_Bypass")})

    t = threading.Thread(target=body)
    t.start()
    t.join()
    return res


def speculation_state():
    """The measuring thread's speculative-store-bypass state and seccomp mode
    (/proc/thread-self/status) and the kernel's global view (sysfs). With
    SSBD on (e.g. forced for every seccomp-filtered process, the kernel's
    default `spec_store_bypass_disable=seccomp`), a load waits for every
    older store's address: the oracle's byte-wise read-modify-write loop is
    exactly that pattern, while register-only and streaming-read code is not
    affected."""
    out = {}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("microcode"):
                out["microcode"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        for line in open("/proc/thread-self/status"):
            key = line.split(":")[0]
            if key in ("Speculation_Store_Bypass", "SpeculationIndirectBranch", "Seccomp",
                       "Seccomp_filters"):
                out[key] = line.split(":", 1)[1].strip()
    except OSError:
        pass
    try:
        out["vulnerabilities_spec_store_bypass"] = open(
            "/sys/devices/system/cpu/vulnerabilities/spec_store_bypass").read().strip()
    except OSError:
        pass
    return out


def proc_stat():
    """Per-CPU jiffies from /proc/stat: {cpu: (total, steal)}."""
    out = {}
    try:
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3:4].isdigit():
                f = line.split()
                v = [int(x) for x in f[1:]]
                out[int(f[0][3:])] = (sum(v), v[7] if len(v) > 7 else 0)
    except (OSError, ValueError):
        pass
    return out


def steal_frac(st0, st1, cpu):
    if cpu not in st0 or cpu not in st1:
        return None
    tot = st1[cpu][0] - st0[cpu][0]
    return round((st1[cpu][1] - st0[cpu][1]) / tot, 4) if tot > 0 else None


def cpu_quota():
    """The CPUs this process may actually use: affinity mask and the cgroup v2
    CPU quota (cpu.max 'quota period'), which can be far below nproc."""
    q = {"nproc": os.cpu_count()}
    try:
        q["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        q["affinity"] = None
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        q["cgroup_cpus"] = None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        q["cgroup_cpus"] = None
    return q


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def node_cpus():
    """{numa node: [allowed logical CPUs]} for this process's affinity set."""
    out = {}
    for c in sorted(os.sched_getaffinity(0)):
        node = cpu_where(c)["numa_node"]
        out.setdefault(node, []).append(c)
    return out



def cpu_ranges(cpus) -> str:
    """[0, 1, 2, 5] -> '0-2,5'."""
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
            continue
        if run:
            out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
        run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def set_process_affinity(cpus) -> None:
    """sched_setaffinity on every thread of this process (the call itself
    only moves the calling thread; threads started later inherit the mask of
    the thread that starts them)."""
    cpus = set(cpus)
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except (OSError, ValueError):
            pass  # a thread that ended meanwhile


def pin_rank(device: int, mode: str = "numa") -> dict:
    """One rank per GPU: pin the whole rank process to the allowed CPUs of its
    GPU's NUMA node (storb_rs_device_numa_node), before the rank allocates or
    starts host threads -- Storb's upload / download tasks (upload.rs:418-420,
    download.rs:505-529) belong on the socket the GPU hangs off: a pageable
    call's host copies cross the socket link otherwise (BENCH_r05 shim_path
    numa: 51.3 vs 60.0 us per (4, 6) 1 MiB encode). Returns what was done;
    `allowed` is the set to restore for the CPU-baseline legs (the reference
    runs unpinned)."""
    allowed = sorted(os.sched_getaffinity(0))
    node = _lib.device_numa_node(device)
    by_node = node_cpus()
    info = {"device": device, "gpu_numa_node": node, "allowed_cpus": cpu_ranges(allowed),
            "mode": mode, "allowed": allowed}
    if mode == "numa" and node is not None and node >= 0 and node in by_node:
        set_process_affinity(by_node[node])
        info["cpus"] = cpu_ranges(by_node[node])
        info["pinned"] = True
    else:
        info["cpus"] = cpu_ranges(allowed)
        info["pinned"] = False
        if mode == "numa":
            info["why_not"] = "GPU node unknown or none of its CPUs in the allowed set"
    return info


@contextlib.contextmanager
def affinity(cpus):
    """Temporarily run this process on `cpus` (every thread), then back."""
    saved = sorted(os.sched_getaffinity(0))
    set_process_affinity(cpus)
    try:
        yield
    finally:
        set_process_affinity(saved)
