"""Rank -> GPU -> NUMA node -> CPU binding (pyeclib_amd/placement.py) on a
faked sysfs tree: KFD topology order, visibility variables, PCI numa_node,
node cpulists and the intersection with the process's own affinity
(each GPU's host traffic on its local NUMA node).
Also the gloo-only bookkeeping reductions bench.py uses (shard.py)."""
import os

import pytest

from pyeclib_amd import placement, shard

# two NUMA nodes; GPUs at 0000:05:00.0 (node 0), 0000:85:00.0 (node 1) and
# 0001:0c:00.0 (node 1); KFD node 0 is the CPU
GPUS = [("0000", 0x05, 0, 0, 0), ("0000", 0x85, 0, 0, 1), ("0001", 0x0C, 0, 0, 1)]


def fake_sysfs(tmp_path, numa=None):
    root = tmp_path / "sys"
    topo = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    (topo / "0").mkdir(parents=True)
    (topo / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\nlocation_id 0\n")
    for n, (dom, bus, dev, fn, node) in enumerate(GPUS, start=1):
        d = topo / str(n)
        d.mkdir()
        loc = bus << 8 | dev << 3 | fn
        d.joinpath("properties").write_text(
            f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {loc}\ndomain {int(dom, 16)}\n"
            f"drm_render_minor {128 + n}\n")
        pci = root / "bus" / "pci" / "devices" / f"{dom}:{bus:02x}:{dev:02x}.{fn}"
        pci.mkdir(parents=True)
        pci.joinpath("numa_node").write_text(f"{node if numa is None else numa}\n")
    for node, cpus in ((0, "0-3,8-9"), (1, "4-7,10-11")):
        d = root / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        d.joinpath("cpulist").write_text(cpus + "\n")
    return str(root)


def test_parse_cpulist():
    assert placement.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert placement.parse_cpulist("") == set()


def test_kfd_order_and_numa(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    assert placement.kfd_gpus(sysfs) == ["0000:05:00.0", "0000:85:00.0", "0001:0c:00.0"]
    r0 = placement.gpu_numa(0, sysfs, env={})
    assert r0["pci"] == "0000:05:00.0" and r0["numa_node"] == 0
    assert r0["node_cpus"] == [0, 1, 2, 3, 8, 9]
    r2 = placement.gpu_numa(2, sysfs, env={})
    assert r2["numa_node"] == 1 and r2["node_cpus"] == [4, 5, 6, 7, 10, 11]
    assert "reason" in placement.gpu_numa(3, sysfs, env={})


def test_visible_devices_remap(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    # HIP device 0 is KFD GPU 2 under ROCR_VISIBLE_DEVICES=2,0
    r = placement.gpu_numa(0, sysfs, env={"ROCR_VISIBLE_DEVICES": "2,0"})
    assert r["pci"] == "0001:0c:00.0"
    # nested: ROCR picks (2, 0), then HIP picks its index 1 -> KFD GPU 0
    r = placement.gpu_numa(0, sysfs, env={"ROCR_VISIBLE_DEVICES": "2,0",
                                          "HIP_VISIBLE_DEVICES": "1"})
    assert r["pci"] == "0000:05:00.0"
    # UUID lists are not resolved: no binding
    assert "reason" in placement.gpu_numa(0, sysfs, env={"HIP_VISIBLE_DEVICES": "GPU-abcd"})


def test_hip_and_cuda_visible_both_set(tmp_path):
    """A launcher that sets HIP_VISIBLE_DEVICES and CUDA_VISIBLE_DEVICES to the
    same list: HIP applies only the former (CUDA_VISIBLE_DEVICES is read only
    when HIP_VISIBLE_DEVICES is unset), so the list is narrowed once."""
    sysfs = fake_sysfs(tmp_path)
    env = {"HIP_VISIBLE_DEVICES": "1,2", "CUDA_VISIBLE_DEVICES": "1,2"}
    assert placement.gpu_numa(0, sysfs, env=env)["pci"] == "0000:85:00.0"
    assert placement.gpu_numa(1, sysfs, env=env)["pci"] == "0001:0c:00.0"
    # CUDA_VISIBLE_DEVICES alone still narrows
    assert placement.gpu_numa(0, sysfs, env={"CUDA_VISIBLE_DEVICES": "2"})["pci"] == "0001:0c:00.0"


def test_bind_intersects_affinity(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    allowed = set(os.sched_getaffinity(0))
    info = placement.bind_to_gpu_numa(1, sysfs, env={}, apply=False)
    want = {4, 5, 6, 7, 10, 11} & allowed
    assert info["cpus_before"] == len(allowed)
    assert info["bound"] == bool(want)
    assert info["cpus"] == (len(want) if want else len(allowed))
    assert info["numa_node"] == 1
    assert set(os.sched_getaffinity(0)) == allowed  # apply=False changed nothing


def test_bind_applies_and_restores(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    before = set(os.sched_getaffinity(0))
    if not ({0, 1, 2, 3, 8, 9} & before):
        pytest.skip("node-0 CPUs of the fake tree not in this process's affinity")
    try:
        info = placement.bind_to_gpu_numa(0, sysfs, env={})
        assert info["bound"]
        assert set(os.sched_getaffinity(0)) == {0, 1, 2, 3, 8, 9} & before
    finally:
        os.sched_setaffinity(0, before)


def test_no_numa_information(tmp_path):
    sysfs = fake_sysfs(tmp_path, numa=-1)
    info = placement.bind_to_gpu_numa(0, sysfs, env={}, apply=False)
    assert info["bound"] is False and info["numa_node"] == -1
    info = placement.bind_to_gpu_numa(0, str(tmp_path / "nothing"), env={}, apply=False)
    assert info["bound"] is False and info["reason"] == "no KFD topology"


def test_device_index_same_device():
    assert shard.device_index(3) == 3
    assert shard.device_index(3, same_device=True) == 0


def test_reductions_without_process_group():
    assert shard.max_over_ranks(2.5) == 2.5
    assert shard.min_over_ranks(1) == 1
    assert shard.sum_over_ranks(7) == 7
