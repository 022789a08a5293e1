"""NUMA placement of the host-side frame rings (SURVEY §8e "host DRAM aggregate").

A GPU worker's frames are DMA'd between its GPU and a shared-memory ring slice (``shm``); on a
two-socket host half the GPUs hang off each socket, and a slice in the other socket's DRAM
makes every H2D/D2H byte cross the socket link.  The worker reports its GPU's node (sysfs,
from the PCI address ``vf_device_pci_bus_id`` gives), and the distributor binds that worker's
slice to the node with ``mbind(MPOL_PREFERRED)`` before any page of it exists.  A tmpfs
(POSIX shm) segment keeps the policy on the shared object, so the pages follow it whichever
process faults them in first (the worker's ``hipHostRegister`` does).

Linux x86-64 system calls through ctypes; anywhere else, or when the kernel refuses (no NUMA
support: ENOSYS), the functions return False / None and placement is left to the kernel.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import platform
from typing import List, Optional

_NR = {"x86_64": {"mbind": 237, "get_mempolicy": 239, "move_pages": 279}}
MPOL_PREFERRED = 1
MPOL_BIND = 2
PAGE = os.sysconf("SC_PAGE_SIZE") if hasattr(os, "sysconf") else 4096

_libc = None


def _syscalls() -> Optional[dict]:
    global _libc
    nr = _NR.get(platform.machine())
    if nr is None:
        return None
    if _libc is None:
        _libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        _libc.syscall.restype = ctypes.c_long
    return nr


def node_count() -> int:
    """Online NUMA nodes (1 where sysfs has none)."""
    try:
        return max(1, len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")
                           and d[4:].isdigit()]))
    except OSError:
        return 1


def pci_numa_node(bus_id: str) -> Optional[int]:
    """NUMA node of PCI device ``bus_id`` ("dddd:bb:dd.f"), None if unknown (-1 in sysfs)."""
    try:
        with open(f"/sys/bus/pci/devices/{bus_id.lower()}/numa_node") as f:
            n = int(f.read().strip())
    except (OSError, ValueError):
        return None
    return n if n >= 0 else None


def gpu_numa_node(device: int) -> Optional[int]:
    """NUMA node of HIP device ``device`` (None if unknown)."""
    from ._lib import device_pci_bus_id
    try:
        return pci_numa_node(device_pci_bus_id(device))
    except Exception:
        return None


def bind(addr: int, nbytes: int, node: int, strict: bool = False) -> bool:
    """Set the memory policy of [addr, addr + nbytes) (page aligned) to ``node``:
    MPOL_PREFERRED (falls back to other nodes when the node is full), MPOL_BIND if
    ``strict``.  Pages that already exist are not moved.  True on success."""
    nr = _syscalls()
    if nr is None or node is None or node < 0 or nbytes <= 0:
        return False
    words = node // 64 + 1
    mask = (ctypes.c_ulong * words)()
    mask[node // 64] = 1 << (node % 64)
    rc = _libc.syscall(nr["mbind"], ctypes.c_void_p(addr), ctypes.c_ulong(nbytes),
                       ctypes.c_int(MPOL_BIND if strict else MPOL_PREFERRED), mask,
                       ctypes.c_ulong(64 * words + 1), ctypes.c_uint(0))
    return rc == 0


def page_nodes(addr: int, nbytes: int, max_pages: int = 4096) -> List[int]:
    """Node of each resident page in [addr, addr + nbytes) (up to ``max_pages`` pages spread
    over the range; negative = errno, e.g. -14 for a page not yet faulted in)."""
    nr = _syscalls()
    if nr is None or nbytes <= 0:
        return []
    npages = (nbytes + PAGE - 1) // PAGE
    step = max(1, npages // max_pages)
    idx = list(range(0, npages, step))
    pages = (ctypes.c_void_p * len(idx))(*[addr + i * PAGE for i in idx])
    status = (ctypes.c_int * len(idx))()
    rc = _libc.syscall(nr["move_pages"], ctypes.c_int(0), ctypes.c_ulong(len(idx)), pages, None, status,
                       ctypes.c_int(0))
    if rc != 0:
        return []
    return list(status)


def node_cpus(node: Optional[int]) -> List[int]:
    """CPUs of NUMA node ``node`` that this process may run on (sysfs cpulist intersected with
    the affinity mask); empty when unknown."""
    if node is None or node < 0:
        return []
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
    except OSError:
        return []
    cpus = set()
    for part in spec.split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    try:
        cpus &= os.sched_getaffinity(0)
    except (AttributeError, OSError):
        pass
    return sorted(cpus)


def pin_thread_to_node(node: Optional[int]) -> bool:
    """Restrict the calling thread to the CPUs of ``node`` (Linux: sched_setaffinity(0) is per
    thread), so the pages it first touches and the memory it streams stay on that socket.
    False (nothing changed) when the node's CPUs are unknown."""
    cpus = node_cpus(node)
    if not cpus:
        return False
    try:
        os.sched_setaffinity(0, cpus)
        return True
    except (AttributeError, OSError):
        return False

