"""Host-side placement of a GPU rank: bind the rank's threads to the CPUs of its GPU's NUMA node.

One process per GPU; on a 2-socket MI355X node four GPUs hang off each socket.  A rank whose
reader threads, pinned staging buffers and out-of-core spill tier live on the far socket pays the
socket interconnect on every PCIe transfer.  ``bind_to_gpu`` restricts the calling process to the
CPUs of the GPU's NUMA node (intersected with the CPUs it may already use), before any large
host buffer is touched, so first-touch places the pinned memory on the local node.  The
reference's counterpart is the scheduler's locality / affinity model for vertex placement
(GraphManager affinity, LocalScheduler); GPU -> rank placement itself stays rank = device.
"""
from __future__ import annotations

import os

SYSFS = "/sys"


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str) -> set:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
    out = set()
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def gpu_numa_node(pci_bus_id: str, sysfs: str = SYSFS) -> int | None:
    """NUMA node of a PCI device ('0000:03:00.0'), None when unknown (-1 in sysfs)."""
    v = _read(os.path.join(sysfs, "bus", "pci", "devices", pci_bus_id.lower(), "numa_node"))
    if v is None:
        return None
    try:
        n = int(v)
    except ValueError:
        return None
    return n if n >= 0 else None


def node_cpus(node: int, sysfs: str = SYSFS) -> set:
    return parse_cpulist(_read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist")) or "")


def pci_address(props) -> str:
    """'dddd:bb:dd.0' of a torch device-properties object (domain / bus / device ids are ints)."""
    bus = getattr(props, "pci_bus_id", None)
    if isinstance(bus, str):
        return bus
    return f"{int(getattr(props, 'pci_domain_id', 0) or 0):04x}:{int(bus or 0):02x}:" \
           f"{int(getattr(props, 'pci_device_id', 0) or 0):02x}.0"


def bind_to_gpu(device_index: int, sysfs: str = SYSFS, apply: bool = True) -> dict:
    """Restrict this process to the CPUs of GPU ``device_index``'s NUMA node.  Returns what was
    decided ({"node", "cpus", "applied"}); never raises (placement is an optimisation)."""
    info = {"node": None, "cpus": 0, "applied": False}
    try:
        import torch
        props = torch.cuda.get_device_properties(device_index)
        node = gpu_numa_node(pci_address(props), sysfs)
    except Exception:  # noqa: BLE001
        return info
    info["node"] = node
    if node is None:
        return info
    cpus = node_cpus(node, sysfs) & set(os.sched_getaffinity(0))
    info["cpus"] = len(cpus)
    if cpus and apply:
        try:
            os.sched_setaffinity(0, cpus)
            info["applied"] = True
        except OSError:
            pass
    return info
