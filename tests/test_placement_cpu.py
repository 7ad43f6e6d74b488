"""Host CPU placement of the ranks of one node (gale/utils: core_groups, numa_slice,
plan_rank_slices), on a fake sysfs of the MI355X box's CPU topology: 2 x EPYC 9575F, 64 cores /
128 threads per socket, node 0 = CPUs 0-63 + 128-191, node 1 = 64-127 + 192-255, SMT siblings
c and c + 128 (profiles/r5_box_topology.txt).

The reference sizes host parallelism per worker JVM (8 workers holding 2 + 4 + 2 executors,
MainTopology.java:25-28,65-66); gale gives each of the 8 GPU ranks its own disjoint slice of
its GPU's NUMA node: 16 physical cores + their 16 SMT siblings, 4 ranks per socket."""

import os

import pytest

from gale.utils import _parse_cpulist, core_groups, numa_slice, plan_rank_slices


def fake_sysfs(root, ncpu=256, half=128):
    for c in range(ncpu):
        d = root / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        core = c % half
        (d / "thread_siblings_list").write_text(f"{core},{core + half}\n")
    return str(root)


NODE0 = set(range(0, 64)) | set(range(128, 192))
NODE1 = set(range(64, 128)) | set(range(192, 256))


def test_core_groups_pairs_siblings(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    g = core_groups(NODE0, sysfs)
    assert len(g) == 64 and g[0] == [0, 128] and g[63] == [63, 191]


def test_eight_ranks_get_disjoint_slices_four_per_node(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    gpu_nodes = [0, 0, 0, 0, 1, 1, 1, 1]  # an 8-GPU MI355X node: GPUs 0-3 on socket 0
    plan = plan_rank_slices(gpu_nodes, {0: NODE0, 1: NODE1}, smt=True, sysfs=sysfs)
    assert len(plan) == 8
    for r, s in enumerate(plan):
        assert len(s) == 32, r
        assert s <= (NODE0 if r < 4 else NODE1)
        cores = {c % 128 for c in s}
        assert len(cores) == 16 and s == cores | {c + 128 for c in cores}  # whole cores
    for i in range(8):
        for j in range(i + 1, 8):
            assert not plan[i] & plan[j], (i, j)
    assert set().union(*plan[:4]) == NODE0 and set().union(*plan[4:]) == NODE1
    # rank 0: cores 0-15 (L3 domains 0-7 and 8-15 on Zen 5) with their siblings
    assert plan[0] == _parse_cpulist("0-15,128-143")
    assert plan[5] == _parse_cpulist("80-95,208-223")


def test_fewer_ranks_get_bigger_slices_and_unknown_node_is_unpinned(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    plan = plan_rank_slices([0, 1], {0: NODE0, 1: NODE1}, smt=True, sysfs=sysfs)
    assert plan == [NODE0, NODE1]
    plan = plan_rank_slices([0, 0, -1], {0: NODE0}, smt=True, sysfs=sysfs)
    assert len(plan[0]) == 64 and len(plan[1]) == 64 and not plan[0] & plan[1]
    assert plan[2] == set()
    # three ranks on one node: 21 cores each (one core left over), still whole cores
    plan = plan_rank_slices([0, 0, 0], {0: NODE0}, smt=True, sysfs=sysfs)
    assert [len(s) for s in plan] == [42, 42, 42]


def test_numa_slice_modes(tmp_path):
    sysfs = fake_sysfs(tmp_path)
    # lowest ids: 16 physical cores, no siblings (bench.py --cpus-per-rank -1 on a 16-CPU quota)
    assert numa_slice(NODE0, 0, 16, smt=False, sysfs=sysfs) == set(range(16))
    # whole cores: 8 cores + siblings
    assert numa_slice(NODE0, 1, 16, smt=True, sysfs=sysfs) == \
        set(range(8, 16)) | set(range(136, 144))
    assert numa_slice(NODE0, 8, 16, smt=True, sysfs=sysfs) == set()  # past the node


@pytest.mark.skipif(not os.path.exists("/sys/devices/system/cpu/cpu0/topology"),
                    reason="no sysfs CPU topology")
def test_real_sysfs_groups_cover_affinity():
    cpus = os.sched_getaffinity(0)
    g = core_groups(cpus)
    assert sorted(c for grp in g for c in grp) == sorted(cpus)
