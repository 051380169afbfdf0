"""deploy/ (Dockerfile + Kubernetes manifests, the counterpart of the reference's
python-scripts/*/model-*.yaml, run.sh and infrastructure/*): every manifest parses,
every streamml command it runs exists, and every flag it passes is accepted by that
command's argument parser (parsed for real with the parser stubbed out at the end)."""
import glob
import os
import shlex

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")


def _containers():
    for path in sorted(glob.glob(os.path.join(DEPLOY, "k8s", "*.yaml"))):
        for doc in yaml.safe_load_all(open(path)):
            if not doc or doc.get("kind") not in ("Job", "Deployment", "StatefulSet", "Pod"):
                continue
            spec = doc["spec"]
            pod = spec["template"]["spec"] if "template" in spec else spec
            for c in pod["containers"]:
                yield os.path.basename(path), c


def _cli_argv(c):
    """The ``python -m streamml.cli`` argv a container runs (entrypoint, torchrun or sh -c)."""
    cmd, args = c.get("command"), [str(a) for a in c.get("args", [])]
    if cmd is None:                      # image ENTRYPOINT = python3 -m streamml.cli
        return args
    if cmd == ["torchrun"]:
        return args[args.index("streamml.cli") + 1:]
    if cmd[:2] == ["sh", "-c"]:
        toks = shlex.split(args[0].replace("$JOB_COMPLETION_INDEX", "0"))
        return toks[toks.index("streamml.cli") + 1:]
    raise AssertionError(f"unexpected command {cmd}")


def test_manifests_parse_and_request_gpus():
    seen = {name for name, _ in _containers()}
    assert {"model-training.yaml", "model-predictions.yaml", "mqtt-broker.yaml", "stream-jobs.yaml",
            "devsim-job.yaml"} <= seen
    gpus = {name: c.get("resources", {}).get("limits", {}).get("amd.com/gpu") for name, c in _containers()}
    assert gpus["model-training.yaml"] == 8 and gpus["model-predictions.yaml"] == 1


@pytest.mark.parametrize("name,container", list(_containers()), ids=lambda v: v if isinstance(v, str) else "")
def test_container_commands_are_valid(name, container, monkeypatch, tmp_path):
    from streamml.cli import __main__ as climain
    argv = _cli_argv(container)
    cmds = climain._commands()
    assert argv[0] in cmds, argv
    if argv[0] == "train":
        from streamml.cli.train import _split
        cfg_path, job, rest = _split(argv[1:])
        assert cfg_path and job["ckpt_dir"]
        return
    # parse the flags with the command's own argparse parser, stopping right after parsing
    import argparse

    class Parsed(Exception):
        pass

    orig = argparse.ArgumentParser.parse_args

    def parse_then_stop(self, args=None, namespace=None):
        ns = orig(self, args, namespace)
        raise Parsed(ns)

    monkeypatch.setattr(argparse.ArgumentParser, "parse_args", parse_then_stop)
    with pytest.raises(Parsed):
        cmds[argv[0]](argv[1:])


def test_deploy_scenario_parses():
    from streamml.mqtt import Scenario
    sc = Scenario.from_xml(os.path.join(DEPLOY, "scenarios", "car-fleet-evaluation.xml"))
    assert (sc.clients, sc.messages_per_client, sc.interval_s, sc.qos, sc.ramp_s) == (25, 40, 5.0, 1, 10.0)
    assert sc.broker == ("hivemq-mqtt", 1883)


def test_devsim_agents_split_the_fleet(tmp_path):
    """--agents/--agent-index give disjoint car-id ranges that cover the fleet."""
    from streamml.kafka import fake_broker
    from streamml.mqtt import MqttBroker, Scenario, simulate
    fake_broker("deploy-split").create_topic("sensor-data", 1)
    with MqttBroker(kafka="fake://deploy-split") as b:
        sc = Scenario().scaled(clients=10, messages=1, interval_s=0.001)
        for a in range(3):
            lo, hi = 10 * a // 3, 10 * (a + 1) // 3
            simulate(sc.scaled(clients=hi - lo), "127.0.0.1", b.port, threads=2, id_offset=lo)
        assert b.flush(5.0)
    keys = sorted(k.decode() for _, k, _ in fake_broker("deploy-split").read("sensor-data", 0, 0))
    assert keys == [f"vehicles/sensor/data/electric-vehicle-{i:05d}" for i in range(10)]
