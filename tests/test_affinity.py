"""CPU: NUMA-local host-thread placement of the engine's entropy pool
(csrc/host/affinity.cpp; SURVEY.md §8(e) "each GPU gets its own host entropy thread
pool, NUMA-local"), run against fake sysfs topologies."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "h264-h265-to-jpeg_amd", "csrc", "host")


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("aff") / "affinity_probe")
    subprocess.check_call(["g++", "-O1", "-std=c++11", "-I", HOST,
                           os.path.join(ROOT, "tools", "affinity_probe", "affinity_probe.cpp"),
                           os.path.join(HOST, "affinity.cpp"), "-o", exe])
    return exe


def _sysfs(tmp_path, nodes, cpu_max=None, pci=None):
    for n, cl in nodes.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True, exist_ok=True)
        (d / "cpulist").write_text(cl + "\n")
    if cpu_max is not None:
        d = tmp_path / "fs" / "cgroup"
        d.mkdir(parents=True, exist_ok=True)
        (d / "cpu.max").write_text(cpu_max + "\n")
    for bus, node in (pci or {}).items():
        d = tmp_path / "bus" / "pci" / "devices" / bus
        d.mkdir(parents=True, exist_ok=True)
        (d / "numa_node").write_text(f"{node}\n")
    return str(tmp_path)


def _plan(probe, root, device, nodes, cpus, quota=0, requested=0, engines=1, pin="1", procs=1):
    env = dict(os.environ, H2J_SYSFS_ROOT=root, H2J_PIN=pin, H2J_LOCAL_PROCS=str(procs))
    out = subprocess.check_output([probe, "plan", str(device), ",".join(map(str, nodes)), cpus, str(quota),
                                   str(requested), str(engines)], env=env, text=True).split()
    kv = dict(x.split("=", 1) for x in out)
    cl = [int(c) for c in kv["cpus"].split(",")] if kv.get("cpus") else []
    return int(kv["threads"]), int(kv["node"]), cl


def test_eight_gpus_two_nodes_disjoint_numa_local(probe, tmp_path):
    root = _sysfs(tmp_path, {0: "0-47,96-143", 1: "48-95,144-191"})
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    seen = set()
    for d in range(8):
        t, n, cl = _plan(probe, root, d, nodes, "0-191")
        assert n == nodes[d]
        assert len(cl) == 24 and t == 24  # 96 CPUs of the node / 4 GPUs of the node
        node_cpus = set(range(0, 48)) | set(range(96, 144)) if n == 0 else set(range(48, 96)) | set(range(144, 192))
        assert set(cl) <= node_cpus
        assert not (set(cl) & seen)
        seen |= set(cl)
    assert len(seen) == 192


def test_quota_bounds_threads_and_is_shared_by_engines(probe, tmp_path):
    root = _sysfs(tmp_path, {0: "0-127"})
    t, _, cl = _plan(probe, root, 0, [0], "0-127", quota=16)
    assert t == 16 and len(cl) == 128  # a 16-CPU cgroup quota on a 128-CPU node
    t, _, _ = _plan(probe, root, 0, [0, 0], "0-127", quota=16, engines=2)
    assert t == 8
    t, _, _ = _plan(probe, root, 0, [0], "0-127")
    assert t == 64  # no quota: capped at 64
    t, _, _ = _plan(probe, root, 0, [0], "0-127", requested=5)
    assert t == 5


def test_quota_is_shared_by_the_ranks_of_a_node(probe, tmp_path):
    # torchrun: 8 rank processes in one cgroup with a 128-CPU quota, 8 GPUs on 2 NUMA nodes
    root = _sysfs(tmp_path, {0: "0-127", 1: "128-255"})
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    for dev in range(8):
        t, n, cl = _plan(probe, root, dev, nodes, "0-255", quota=128, procs=8)
        assert t == 16 and n == nodes[dev] and len(cl) == 32
    # LOCAL_WORLD_SIZE (torchrun) is the fallback for H2J_LOCAL_PROCS
    env = dict(os.environ, H2J_SYSFS_ROOT=root, H2J_PIN="1", LOCAL_WORLD_SIZE="4")
    env.pop("H2J_LOCAL_PROCS", None)
    out = subprocess.check_output([probe, "plan", "0", ",".join(map(str, nodes)), "0-255", "128", "0", "1"],
                                  env=env, text=True)
    assert out.startswith("threads=32 ")


def test_mask_outside_node_and_unknown_topology(probe, tmp_path):
    root = _sysfs(tmp_path, {0: "0-7", 1: "8-15"})
    # the process may only run on node 1's CPUs, the GPU sits on node 0: use the mask
    t, _, cl = _plan(probe, root, 0, [0, 1], "8-15")
    assert cl == list(range(8, 12)) and t == 4  # unknown locality: split between the 2 devices
    t, n, cl = _plan(probe, root, 1, [-1, -1], "0-15")
    assert n == -1 and cl == list(range(8, 16))
    t, _, cl = _plan(probe, root, 0, [0], "0-7", pin="0")
    assert cl == [] and t == 8  # H2J_PIN=0: sized, not pinned


def test_sysfs_readers(probe, tmp_path):
    root = _sysfs(tmp_path, {0: "0-3"}, cpu_max="1600000 100000", pci={"0000:c5:00.0": 1})
    env = dict(os.environ, H2J_SYSFS_ROOT=root)
    out = subprocess.check_output([probe, "sysfs", "0000:C5:00.0"], env=env, text=True).split()
    assert out == ["numa=1", "quota=16"]
    (tmp_path / "fs" / "cgroup" / "cpu.max").write_text("max 100000\n")
    out = subprocess.check_output([probe, "sysfs", "0000:00:00.0"], env=env, text=True).split()
    assert out == ["numa=-1", "quota=0"]
