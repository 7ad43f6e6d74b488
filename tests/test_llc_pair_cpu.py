"""L3-domain pairing of the in-process broker's connection threads with the engine's source
threads (csrc/kafka/llc_pair.cpp, gale/llc_pair.h), on a fake two-domain sysfs topology: source
threads are pinned round robin to the domains of their mask, and a broker thread that looks up its
peer's registered port is pinned to the same domain."""

import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fake_sysfs(tmp_path, cpus):
    half = len(cpus) // 2
    doms = [cpus[:half], cpus[half:]]
    for d in doms:
        lst = ",".join(map(str, d))
        for c in d:
            p = tmp_path / f"cpu{c}" / "cache" / "index3"
            p.mkdir(parents=True)
            (p / "shared_cpu_list").write_text(lst + "\n")
    return doms


def test_source_and_broker_threads_share_an_l3_domain(tmp_path):
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs two CPUs")
    doms = _fake_sysfs(tmp_path, cpus)
    code = textwrap.dedent("""
        import json, os, threading
        from gale._native import native
        C = native()
        out = {}
        def source(name, port):
            out[name] = C.llc_pin_self_next_domain()
            out[name + "_cpus"] = sorted(os.sched_getaffinity(0))
            C.llc_register_local_port(port)
        def broker(name, port):
            out[name] = C.llc_pin_self_for_peer(port)
            out[name + "_cpus"] = sorted(os.sched_getaffinity(0))
        for args in (("s1", 40001), ("s2", 40002)):
            t = threading.Thread(target=source, args=args); t.start(); t.join()
        for args in (("b1", 40001), ("b2", 40002), ("b3", 40003)):
            t = threading.Thread(target=broker, args=args); t.start(); t.join()
        out["main_cpus"] = sorted(os.sched_getaffinity(0))
        print(json.dumps(out))
    """)
    env = dict(os.environ, GALE_SYSFS_CPU=str(tmp_path), GALE_LLC_PAIR="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # round robin over the two domains, named by their lowest CPU
    assert {out["s1"], out["s2"]} == {doms[0][0], doms[1][0]}
    assert out["s1_cpus"] in doms and out["s2_cpus"] in doms
    assert out["s1_cpus"] != out["s2_cpus"]
    # each broker thread follows its peer's domain; an unknown port leaves it unpinned
    assert out["b1"] and out["b1_cpus"] == out["s1_cpus"]
    assert out["b2"] and out["b2_cpus"] == out["s2_cpus"]
    assert not out["b3"] and out["b3_cpus"] == cpus
    assert out["main_cpus"] == cpus  # (per-thread affinity only)


def test_pairing_off_and_single_domain_are_no_ops(tmp_path):
    cpus = sorted(os.sched_getaffinity(0))
    p = tmp_path / "one"
    for c in cpus:
        d = p / f"cpu{c}" / "cache" / "index3"
        d.mkdir(parents=True)
        (d / "shared_cpu_list").write_text(",".join(map(str, cpus)) + "\n")
    code = ("from gale._native import native; C = native(); "
            "print(C.llc_pin_self_next_domain())")
    for env_extra, sysfs in (({"GALE_LLC_PAIR": "1"}, str(p)), ({"GALE_LLC_PAIR": "0"}, None)):
        env = dict(os.environ, **env_extra)
        if sysfs:
            env["GALE_SYSFS_CPU"] = sysfs
        r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.strip().splitlines()[-1] == "-1"
