"""Rank placement on the host: bind a rank's CPU affinity to its GPU's NUMA node.

One process per GPU (bench.py, tools/swift_mix.py).  The host-resident and
Swift-mix legs move ~50 GB/s per GPU between pinned host memory and the GPU
(SURVEY §7(f), §8(e)); with 8 GPUs that meets the host's DRAM, so each rank's
threads -- and the pinned buffers they first touch -- belong on the NUMA node
the GPU's PCIe root hangs off.

The GPU of local rank r is found WITHOUT touching the GPU (binding must
happen before the HIP runtime starts its threads, which inherit the mask, and
nothing here may initialise the device):
  1. HIP's device order is the KFD topology order of the GPU nodes
     (/sys/class/kfd/kfd/topology/nodes/N/properties: `simd_count` > 0 marks a
     GPU; `domain` and `location_id` = bus << 8 | device << 3 | function give
     its PCI address), narrowed by ROCR_VISIBLE_DEVICES, then
     HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (index lists);
  2. the PCI device's `numa_node` (/sys/bus/pci/devices/<addr>/numa_node);
  3. that node's CPUs (/sys/devices/system/node/node<n>/cpulist), intersected
     with the CPUs this process may already use (a cgroup cpuset, a launcher's
     mask).  An empty intersection, a node of -1 or any missing file leaves
     the affinity unchanged and says why.
Every path is under a `sysfs` root, so tests run it on a faked tree.
"""
from __future__ import annotations

import os


def parse_cpulist(text: str) -> set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
    cpus: set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.update(range(int(lo), int(hi) + 1))
        else:
            cpus.add(int(part))
    return cpus


def _read(path: str) -> str | None:
    try:
        with open(path) as fh:
            return fh.read()
    except OSError:
        return None


def kfd_gpus(sysfs: str = "/sys") -> list[str]:
    """PCI addresses ('dddd:bb:dd.f') of the GPUs in KFD topology order."""
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted((int(n) for n in os.listdir(base) if n.isdigit()))
    except OSError:
        return []
    out = []
    for n in nodes:
        text = _read(os.path.join(base, str(n), "properties"))
        if text is None:
            continue
        props = {}
        for line in text.splitlines():
            f = line.split()
            if len(f) == 2 and f[1].lstrip("-").isdigit():
                props[f[0]] = int(f[1])
        if props.get("simd_count", 0) <= 0 or "location_id" not in props:
            continue
        loc, dom = props["location_id"], props.get("domain", 0)
        out.append(f"{dom:04x}:{loc >> 8 & 0xFF:02x}:{loc >> 3 & 0x1F:02x}.{loc & 7:x}")
    return out


def _visible(order: list, env: dict) -> list:
    """Narrow a device list by the runtime's visibility variables (index
    lists only; a UUID list -- or an index out of range -- gives [] and the
    caller does not bind).  ROCR_VISIBLE_DEVICES applies first (the ROCr
    runtime's filter), then HIP_VISIBLE_DEVICES; HIP honours
    CUDA_VISIBLE_DEVICES only when HIP_VISIBLE_DEVICES is unset, so the two
    never narrow the list twice."""
    hip = env.get("HIP_VISIBLE_DEVICES")
    hip_set = hip is not None and hip.strip() != ""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES" if hip_set else "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None or v.strip() == "":
            continue
        picked = []
        for tok in v.split(","):
            tok = tok.strip()
            if not tok.isdigit() or int(tok) >= len(order):
                return []
            picked.append(order[int(tok)])
        order = picked
    return order


def gpu_numa(local_rank: int, sysfs: str = "/sys", env: dict | None = None) -> dict:
    """{'pci', 'numa_node', 'node_cpus'} for the GPU a rank uses, or
    {'reason'} when it cannot be determined."""
    env = os.environ if env is None else env
    gpus = kfd_gpus(sysfs)
    if not gpus:
        return {"reason": "no KFD topology"}
    gpus = _visible(gpus, env)
    if not 0 <= local_rank < len(gpus):
        return {"reason": f"device {local_rank} not in the visible GPU list ({len(gpus)})"}
    pci = gpus[local_rank]
    node_txt = _read(os.path.join(sysfs, "bus", "pci", "devices", pci, "numa_node"))
    if node_txt is None:
        return {"pci": pci, "reason": "no numa_node for the PCI device"}
    node = int(node_txt.strip())
    if node < 0:
        return {"pci": pci, "numa_node": node, "reason": "device reports no NUMA node"}
    cpus_txt = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
    if cpus_txt is None:
        return {"pci": pci, "numa_node": node, "reason": "no cpulist for the node"}
    return {"pci": pci, "numa_node": node, "node_cpus": sorted(parse_cpulist(cpus_txt))}


def bind_to_gpu_numa(local_rank: int, sysfs: str = "/sys", env: dict | None = None,
                     apply: bool = True) -> dict:
    """Restrict this process's CPU affinity to its GPU's NUMA node (call it
    before anything initialises the GPU).  Returns what was done: pci,
    numa_node, cpus (the count now allowed) and bound (bool), or a reason."""
    info = gpu_numa(local_rank, sysfs, env)
    allowed = set(os.sched_getaffinity(0))
    info["cpus_before"] = len(allowed)
    node_cpus = set(info.pop("node_cpus", []))
    want = node_cpus & allowed
    if not want:
        info.setdefault("reason", "node CPUs outside this process's affinity")
        info.update(bound=False, cpus=len(allowed))
        return info
    if apply and want != allowed:
        os.sched_setaffinity(0, want)
    info.update(bound=True, cpus=len(want))
    return info
