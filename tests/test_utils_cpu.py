"""Typed node config (utils.config), structured JSON logs (utils.logging) and the
profiling hooks (utils.profiling) -- SURVEY.md 5.1, 5.5, 5.6."""
import io
import json
import os

import pytest
import torch

from shai_amd.utils import profiling
from shai_amd.utils.config import load_node_config
from shai_amd.utils.logging import configure, get_logger

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_node_yaml_validates_and_env_overrides():
    c = load_node_config(os.path.join(ROOT, "config", "node.yaml"),
                         environ={"SHAI_NODE__ROUTER__PORT": "9100", "SHAI_NODE__FAILOVER__THRESHOLD": "0.25"})
    assert c.router.port == 9100 and c.failover.threshold == 0.25
    names = [d.name for d in c.deployments]
    assert "sd21" in names and "mistral" in names
    mistral = next(d for d in c.deployments if d.name == "mistral")
    assert mistral.tp == 2 and mistral.env["APP"] == "mistral-mi355x"
    assert isinstance(next(d for d in c.deployments if d.name == "sd21").env["NUM_OF_RUNS_INF"], str)


@pytest.mark.parametrize("bad", [
    "deployments: [{name: a, module: m, tp: 3}]",                          # TP not 1/2/4/8
    "gpus: [0, 1]\ndeployments: [{name: a, module: m, replicas: 3}]",       # more GPUs than inventory
    "deployments: [{name: a, module: m}, {name: a, module: m}]",            # duplicate names
    "router: {policy: random}",
    "deployments: [{name: a, module: m, autoscale: {target_per_replica: 10, min: 5, max: 2}}]",
])
def test_node_config_rejects(bad):
    with pytest.raises(Exception):
        load_node_config(text=bad, environ={})


def test_json_logs_carry_identity_and_extras(monkeypatch):
    monkeypatch.setenv("APP", "sd21-mi355x")
    monkeypatch.setenv("POD_NAME", "gpu3")
    buf = io.StringIO()
    configure(fmt="json", level="INFO", stream=buf)
    try:
        get_logger("engine").info("step done", extra={"step_ms": 12.5, "batch": 8})
        rec = json.loads(buf.getvalue().strip().splitlines()[-1])
        assert rec["msg"] == "step done" and rec["level"] == "INFO" and rec["logger"] == "shai.engine"
        assert rec["app"] == "sd21-mi355x" and rec["pod"] == "gpu3"
        assert rec["step_ms"] == 12.5 and rec["batch"] == 8
    finally:
        configure(fmt="text")


def test_profiling_ranges_and_session(tmp_path):
    was = profiling.enabled()
    # disabled: pure no-op
    profiling.enable(False)
    with profiling.range_("x"):
        pass
    profiling.enable(True, str(tmp_path))
    try:
        with profiling.profile_session("unit"):
            with profiling.range_("inner"):
                torch.ones(8).sum()
        files = [f for f in os.listdir(tmp_path) if f.startswith("unit-")]
        assert files, os.listdir(tmp_path)
        trace = json.load(open(tmp_path / files[0]))
        names = {e.get("name") for e in trace.get("traceEvents", [])}
        assert "inner" in names and "unit" in names
        t = profiling.StepTimer()
        with t.phase("a"):
            pass
        assert t.report()["a"]["calls"] == 1
    finally:
        profiling.enable(was, "")
