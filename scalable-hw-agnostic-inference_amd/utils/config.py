"""Typed node / deployment configuration.

The reference's "flag system" is environment variables in Deployment manifests
(SURVEY.md 2.12), ConfigMaps (`/vllm_config.yaml`, `models.json`) and per-pool
Karpenter / KEDA YAML.  Here one YAML file (``config/node.yaml``) describes the whole
8x MI355X node and is validated by these pydantic models before anything is launched:

* ``NodeConfig``: GPU inventory, router, autoscaler / failover / health intervals and the
  list of ``Deployment`` units (model server module, DP replicas, TP degree, env).
* Values can be overridden from the environment without editing the file:
  ``SHAI_NODE__ROUTER__PORT=9000`` -> ``router.port = 9000`` (``__`` separates levels;
  values are parsed as YAML scalars).
* Deployment ``env`` keeps the reference's variable names (``APP``, ``MODEL_ID``,
  ``NUM_OF_RUNS_INF``, ``MAX_NEW_TOKENS``, ``HEIGHT``/``WIDTH``/``MAX_SEQ_LEN``...), which the
  servers read through ``serving.common.ServerEnv``.
* TP degrees are checked against xGMI-friendly sizes (1/2/4/8) and the GPU inventory, so
  a config that cannot be placed fails at load time instead of at launch.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import yaml
from pydantic import BaseModel, Field, field_validator, model_validator


class RouterConfig(BaseModel):
    port: int = 8080
    policy: str = "weighted"
    sticky: bool = False
    health_interval_s: float = 10.0

    @field_validator("policy")
    @classmethod
    def _policy(cls, v):
        ok = {"weighted", "round_robin", "least_outstanding"}
        if v not in ok:
            raise ValueError(f"router.policy {v!r} not in {sorted(ok)}")
        return v


class FailoverConfig(BaseModel):
    threshold: float = Field(0.5, ge=0.0, le=1.0)
    interval_s: float = 300.0
    fallback_hold_s: float = 60.0


class HealthConfig(BaseModel):
    interval_s: float = 10.0
    max_temp_c: float = 105.0
    hang_timeout_s: float = 120.0


class AutoscaleConfig(BaseModel):
    target_per_replica: float = Field(gt=0)
    min: int = Field(1, ge=0)
    max: int = Field(8, ge=1)
    window_s: float = 60.0
    scale_down_stabilization_s: float = 300.0

    @model_validator(mode="after")
    def _bounds(self):
        if self.min > self.max:
            raise ValueError(f"autoscale.min {self.min} > max {self.max}")
        return self


class Deployment(BaseModel):
    name: str
    module: str
    replicas: int = Field(1, ge=0)
    tp: int = 1
    pool: str = "cost"
    env: Dict[str, str] = Field(default_factory=dict)
    autoscale: Optional[AutoscaleConfig] = None
    cost_per_hour: float = 1.0
    max_throughput: float = 1.0
    latency_s: float = 1.0

    @field_validator("tp")
    @classmethod
    def _tp(cls, v):
        if v not in (1, 2, 4, 8):
            raise ValueError(f"tp={v}: TP groups are 1, 2, 4 or 8 GPUs of one xGMI node")
        return v

    @field_validator("env", mode="before")
    @classmethod
    def _env(cls, v):
        return {str(k): str(x) for k, x in (v or {}).items()}

    @field_validator("pool")
    @classmethod
    def _pool(cls, v):
        if v not in ("cost", "capacity"):
            raise ValueError(f"pool {v!r} must be 'cost' or 'capacity'")
        return v


class NodeConfig(BaseModel):
    gpus: List[int] = Field(default_factory=lambda: list(range(8)))
    router: RouterConfig = Field(default_factory=RouterConfig)
    autoscale_interval_s: float = 30.0
    failover: FailoverConfig = Field(default_factory=FailoverConfig)
    health: HealthConfig = Field(default_factory=HealthConfig)
    deployments: List[Deployment] = Field(default_factory=list)

    @model_validator(mode="after")
    def _placement(self):
        names = [d.name for d in self.deployments]
        if len(set(names)) != len(names):
            raise ValueError(f"duplicate deployment names: {names}")
        need = sum(d.replicas * d.tp for d in self.deployments)
        if need > len(self.gpus):
            raise ValueError(f"deployments need {need} GPUs at start, inventory has {len(self.gpus)}")
        for d in self.deployments:
            if d.tp > len(self.gpus):
                raise ValueError(f"{d.name}: tp={d.tp} exceeds the {len(self.gpus)}-GPU inventory")
        return self

    def as_dict(self) -> dict:
        return self.model_dump()


def _set_path(d: dict, path: List[str], value):
    for k in path[:-1]:
        d = d.setdefault(k, {})
    d[path[-1]] = value


def apply_env_overrides(raw: dict, environ=None, prefix: str = "SHAI_NODE__") -> dict:
    environ = os.environ if environ is None else environ
    for k, v in environ.items():
        if k.startswith(prefix):
            path = [p.lower() for p in k[len(prefix):].split("__") if p]
            if path:
                _set_path(raw, path, yaml.safe_load(v))
    return raw


def load_node_config(path: Optional[str] = None, text: Optional[str] = None, environ=None) -> NodeConfig:
    if text is None:
        with open(path) as f:
            text = f.read()
    raw = yaml.safe_load(text) or {}
    return NodeConfig.model_validate(apply_env_overrides(raw, environ))
