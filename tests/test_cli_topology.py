"""CLI / config / topology lifecycle (R1, R2, R3, §5.6): positional contract, precedence
CLI > env > TOML > defaults, the registry's AlreadyAlive / NotAlive semantics, a stub topology
run with an embedded broker, and weight files."""

import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from gale.cli import parse_topology_args
from gale.config import GaleConfig, from_sources
from gale.models import get_model, init_params
from gale.models.weights_io import load_params, save_params
from gale.topology import AlreadyAliveError, NotAliveError, Registry, run_topology

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_positional_contract_and_reference_defaults():
    cfg = parse_topology_args(["topo", "in-topic", "out-topic"])
    assert (cfg.topology_name, cfg.input_topic, cfg.output_topic) == ("topo", "in-topic",
                                                                      "out-topic")
    # MainTopology.java:25-28 constants and :101-103 / :113 Kafka settings
    assert (cfg.workers, cfg.source_parallelism, cfg.sink_parallelism) == (8, 2, 2)
    assert cfg.start_offset == "latest" and cfg.acks == 1 and cfg.duration == 3600
    assert cfg.on_error == "null" and cfg.sink_mode == "async"
    with pytest.raises(SystemExit):
        parse_topology_args(["only-two", "args"])  # the reference throws AIOOBE here


def test_precedence_cli_env_toml(tmp_path):
    toml = tmp_path / "g.toml"
    toml.write_text('[gale]\nmax_batch = 64\nmodel = "lenet5"\nacks = -1\n')
    cfg = from_sources(cli={"max_batch": 32}, env={"GALE_MODEL": "resnet50", "GALE_STUB": "1"},
                       toml_path=str(toml))
    assert cfg.max_batch == 32 and cfg.model == "resnet50" and cfg.acks == -1 and cfg.stub
    cfg2 = parse_topology_args(["t", "a", "b", "--config", str(toml), "--no-use-graph",
                                "--sink-mode", "fire-and-forget"])
    assert cfg2.max_batch == 64 and not cfg2.use_graph and cfg2.sink_mode == "fire-and-forget"
    with pytest.raises(ValueError):
        from_sources(cli={"bogus": 1}, env={})
    with pytest.raises(ValueError):
        from_sources(cli={"dtype": "int4"}, env={})


def test_registry_semantics(tmp_path):
    r = Registry(str(tmp_path))
    r.register("a", {"x": 1})
    assert r.get("a")["x"] == 1 and [x["name"] for x in r.list()] == ["a"]
    r2 = Registry(str(tmp_path))
    with pytest.raises(AlreadyAliveError):
        r2.register("a", {})
    r.unregister("a")
    assert r.get("a") is None
    with pytest.raises(NotAliveError):
        r.kill("a")


def test_run_topology_stub_with_embedded_broker(tmp_path):
    from gale._native import native

    K = native().kafka
    cfg = GaleConfig(topology_name="lifecycle", input_topic="in", output_topic="out",
                     bootstrap="127.0.0.1:0", stub=True, duration=30, metrics_interval=0,
                     registry_dir=str(tmp_path), start_offset="earliest")
    # embedded broker on an ephemeral port: start it here and point the topology at it
    b = K.Broker()
    b.start()
    b.create_topic("in", 1)
    b.create_topic("out", 1)
    cfg.bootstrap = f"127.0.0.1:{b.port}"
    from gale._native import native as n

    for i in range(5):
        b.append("in", 0, [n().encode_instances(np.full((1, 32, 32, 3), i / 5, np.float32))])
    stop = threading.Event()
    res = {}
    th = threading.Thread(target=lambda: res.update(run_topology(cfg, stop, False)))
    th.start()
    deadline = time.time() + 20
    while time.time() < deadline and b.log_end("out", 0) < 5:
        time.sleep(0.05)
    assert Registry(str(tmp_path)).get("lifecycle") is not None
    stop.set()
    th.join(30)
    assert res["records_out"] == 5 and b.log_end("out", 0) == 5
    assert Registry(str(tmp_path)).get("lifecycle") is None
    b.stop()


def test_cli_subprocess_kill(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    port = 19000 + os.getpid() % 1000
    p = subprocess.Popen([sys.executable, "-m", "gale", "clitopo", "in", "out", "--stub",
                          "--embedded-broker", "--bootstrap", f"127.0.0.1:{port}",
                          "--registry-dir", str(tmp_path), "--metrics-interval", "0"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        deadline = time.time() + 60
        listed = []
        while time.time() < deadline and not listed:
            out = subprocess.run([sys.executable, "-m", "gale", "list", "--registry-dir",
                                  str(tmp_path)], cwd=ROOT, env=env, capture_output=True,
                                 text=True).stdout
            listed = [json.loads(x) for x in out.splitlines() if x.strip()]
            time.sleep(0.2)
        assert listed and listed[0]["name"] == "clitopo"
        time.sleep(0.5)
        rc = subprocess.run([sys.executable, "-m", "gale", "kill", "clitopo", "--wait-secs",
                             "20", "--registry-dir", str(tmp_path)], cwd=ROOT, env=env).returncode
        assert rc == 0
        assert p.wait(30) == 0
    finally:
        if p.poll() is None:
            p.kill()


def test_weights_roundtrip(tmp_path):
    net = get_model("lenet5")
    params = init_params(net, seed=3)
    for ext in ("npz", "safetensors"):
        path = str(tmp_path / f"w.{ext}")
        save_params(params, path)
        back = load_params(path, net)
        assert set(back) == set(params)
        for k in params:
            np.testing.assert_array_equal(back[k].numpy(), params[k].numpy())
    bad = {k: v for k, v in params.items() if k != "fc3.bias"}
    save_params(bad, str(tmp_path / "bad.npz"))
    with pytest.raises(ValueError):
        load_params(str(tmp_path / "bad.npz"), net)


def test_profile_flag_wraps_run_in_rocprofv3():
    from gale.cli import parse_topology_args, profile_command

    argv = ["t1", "in", "out", "--profile", "/tmp/p", "--model", "lenet5"]
    cfg = parse_topology_args(argv)
    cmd = profile_command(cfg, argv)
    assert cmd[0] == "rocprofv3" and "--marker-trace" in cmd and "--kernel-trace" in cmd
    dd = cmd.index("--")
    assert cmd[dd + 1].endswith("python3") or "python" in cmd[dd + 1]
    assert cmd[dd + 2:dd + 4] == ["-m", "gale"]
    assert "--profile" not in cmd[dd:] and cmd[-1] == "--trace"
    assert cmd[cmd.index("-d") + 1] == "/tmp/p"
    assert parse_topology_args(cmd[dd + 4:]).trace is True


def test_metrics_http_endpoint_prometheus_and_json():
    """--metrics-port: Storm UI's per-component numbers on demand (Prometheus text + JSON)."""
    import json as _json
    import re as _re
    import urllib.request

    from gale.config import GaleConfig
    from gale.engine import Engine
    from gale.metrics import MetricsServer
    from gale._native import native

    C = native()
    b = C.kafka.Broker()
    b.start()
    try:
        b.create_topic("in", 2)
        b.create_topic("out", 1)
        for i in range(6):
            b.append("in", i % 2, [C.encode_instances(np.zeros((1, 32, 32, 3), np.float32))])
        cfg = GaleConfig(topology_name="m", input_topic="in", output_topic="out", stub=True,
                         bootstrap=f"127.0.0.1:{b.port}", start_offset="earliest", replicas=2)
        eng = Engine(cfg, max_records=6)
        eng.start()
        assert eng.wait(30)
        srv = MetricsServer(eng, 0, labels={"topology": "m", "rank": 0}).start()
        try:
            txt = urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/metrics").read().decode()
            js = _json.loads(urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/stats").read())
        finally:
            srv.stop()
            eng.stop()
    finally:
        b.stop()
    assert 'gale_records_out{rank="0",topology="m"} 6' in txt
    assert len(_re.findall(r'^gale_replica_alive\{', txt, _re.M)) == 2
    assert len(_re.findall(r'^gale_partition_lag\{', txt, _re.M)) == 2
    names = [ln.split()[2] for ln in txt.splitlines() if ln.startswith("# TYPE")]
    assert len(names) == len(set(names))  # one family block per metric
    assert js["stats"]["records_out"] == 6 and len(js["replicas"]) == 2
