"""Best-effort NUMA placement: bind the calling process to the CPUs of the NUMA node that hosts a
GPU, so that pinned ingest buffers (first-touch) live next to that GPU's PCIe root complex.

On an 8×MI355X node every rank streams ~50 GB/s of records over its own PCIe link; with the
buffers on the wrong socket that traffic would cross the inter-socket fabric as well.
"""

from __future__ import annotations

import logging
import os
from typing import List, Optional

logger = logging.getLogger(__name__)


def _parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def gpu_numa_node(device_index: int) -> Optional[int]:
    try:
        import torch

        props = torch.cuda.get_device_properties(device_index)
        bus = getattr(props, "pci_bus_id", None)
        dom = getattr(props, "pci_domain_id", 0) or 0
        dev = getattr(props, "pci_device_id", 0) or 0
        if bus is None:
            return None
        path = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.0/numa_node"
        with open(path) as fh:
            node = int(fh.read().strip())
        return node if node >= 0 else None
    except Exception:  # noqa: BLE001 - best effort
        return None


def bind_to_gpu_numa(device_index: int) -> Optional[int]:
    """Restrict this process to the CPUs of the GPU's NUMA node; returns the node or None."""
    node = gpu_numa_node(device_index)
    if node is None:
        return None
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            cpus = set(_parse_cpulist(fh.read())) & os.sched_getaffinity(0)
        if cpus:
            os.sched_setaffinity(0, cpus)
            return node
    except Exception as e:  # noqa: BLE001
        logger.debug("NUMA binding failed: %s", e)
    return None
