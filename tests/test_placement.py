"""Host placement of the multi-GPU path (DESIGN.md section 7, round-5 VERDICT
item 3), on the CPU: the library reads each GPU's NUMA node from sysfs,
pins its shard workers and the device's pack-pool helpers to that node's
CPUs (within the process's own affinity), and splits a node's CPUs among the
pack pools of its GPUs.  A mocked sysfs tree stands in for an 8-GPU,
two-socket host; the pinning mechanism itself runs on this machine's CPUs."""
import ctypes
import os

import pytest


@pytest.fixture(scope="module")
def tlib():
    from hsverify import _lib
    lib = _lib.load_test()
    if lib is None:
        pytest.skip("libhsv_test.so not built")
    return lib


def fake_sysfs(root, gpus, nodes):
    """gpus: {bdf: numa_node}; nodes: {node: cpulist}"""
    for bdf, node in gpus.items():
        d = os.path.join(root, "bus", "pci", "devices", bdf)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "numa_node"), "w") as f:
            f.write(f"{node}\n")
    for node, cpus in nodes.items():
        d = os.path.join(root, "devices", "system", "node", f"node{node}")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "cpulist"), "w") as f:
            f.write(cpus + "\n")
    return root


def plan(tlib, root, bdfs, allowed, pack_default=11):
    n = len(bdfs)
    node, ncpu, pack = ((ctypes.c_int * n)() for _ in range(3))
    got = tlib.hsv_test_numa_plan(str(root).encode(), ",".join(bdfs).encode(), allowed.encode(), pack_default,
                                  node, ncpu, pack, n)
    assert got == n
    return list(node), list(ncpu), list(pack)


# an MI355X node: 8 GPUs, four behind each socket (lspci bus ids as HIP reports them)
BDFS = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
        "0000:85:00.0", "0000:95:00.0", "0000:E5:00.0", "0000:F5:00.0"]


def test_eight_gpus_two_sockets(tlib, tmp_path):
    root = fake_sysfs(tmp_path, {b.lower(): (0 if i < 4 else 1) for i, b in enumerate(BDFS)},
                      {0: "0-63,128-191", 1: "64-127,192-255"})
    node, ncpu, pack = plan(tlib, root, BDFS, "0-255")
    assert node == [0] * 4 + [1] * 4
    assert ncpu == [128] * 8            # every GPU's threads on its own socket's 128 CPUs
    assert pack == [11] * 8             # 128 / 4 GPUs = 32 CPUs per GPU: the full 11 helpers each


def test_node_cpus_shared_among_its_gpus(tlib, tmp_path):
    """A cgroup that leaves 16 CPUs per node: four GPUs on a node get 3 helpers
    each (16 / 4 - 1: one CPU of each share for the GPU's shard worker)."""
    root = fake_sysfs(tmp_path, {b.lower(): (0 if i < 4 else 1) for i, b in enumerate(BDFS)},
                      {0: "0-63", 1: "64-127"})
    node, ncpu, pack = plan(tlib, root, BDFS, "0-15,64-79")
    assert node == [0] * 4 + [1] * 4 and ncpu == [16] * 8 and pack == [3] * 8


def test_unknown_or_excluded_nodes_stay_unpinned(tlib, tmp_path):
    """numa_node -1 (one NUMA node, or no information), a missing sysfs entry,
    and a node outside the process's affinity: no pinning, the default pool."""
    root = fake_sysfs(tmp_path, {"0000:05:00.0": 0, "0000:15:00.0": -1, "0000:85:00.0": 1},
                      {0: "0-3", 1: "4-7"})
    node, ncpu, pack = plan(tlib, root, ["0000:05:00.0", "0000:15:00.0", "0000:85:00.0", "0000:aa:00.0"], "0-3",
                            pack_default=5)
    assert node == [0, -1, 1, -1]
    assert ncpu == [4, 0, 0, 0]          # node 1 exists but none of its CPUs is allowed
    assert pack == [3, 5, 5, 5]          # node 0's 4 CPUs: 3 helpers + the worker; the rest: default


def test_malformed_cpulist_is_rejected(tlib, tmp_path):
    root = fake_sysfs(tmp_path, {"0000:05:00.0": 0}, {0: "3-1"})
    node, ncpu, _ = plan(tlib, root, ["0000:05:00.0"], "0-7")
    assert node == [-1] and ncpu == [0]
    assert tlib.hsv_test_numa_plan(str(root).encode(), b"0000:05:00.0", b"x-y", 1, None, None, None, 0) < 0


def test_worker_threads_are_pinned_to_the_node(tlib):
    """The pinning the shard workers and pack helpers use: a new thread bound
    to a node's CPUs reports exactly those CPUs as its affinity."""
    mine = sorted(os.sched_getaffinity(0))
    want = mine[-2:] if len(mine) >= 2 else mine
    cpus = (ctypes.c_int * 64)()
    n = tlib.hsv_test_pinned_thread_cpus(",".join(map(str, want)).encode(), cpus, 64)
    assert n == len(want) and list(cpus[:n]) == want
    assert sorted(os.sched_getaffinity(0)) == mine  # the caller's own thread is untouched
