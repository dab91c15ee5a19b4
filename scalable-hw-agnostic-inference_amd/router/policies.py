"""Traffic-distribution policies and the reference's weight formulas.

The reference distributes traffic across "deployment units" D_i with an ALB
``actions.weighted-routing`` forward config (sd21-weighted-routing-ing.yaml:19-20)
or one round-robin Service (sd21-equal-routing-ing.yaml), and documents the
weight math in README.md:158-292.  Here the units are local replicas (one per
GPU or TP group) and the same formulas drive an in-process router:

* :func:`efficiency_weights`  w_i = (T_i / (C_i L_i)) A_i / sum_j (T_j / (C_j L_j)) A_j   (README eq. 1)
* :func:`cost_weights`        w_i = (C_i / L_i) / sum_j (C_j / L_j)                       (Option 1, as printed)
* :func:`capacity_weights`    w_i = A_i / sum_j A_j                                       (Option 2)
* :func:`adjusted_throughput` min(sum(T_max)/N, T_max_i)                                 (Option 2 targets)
* :func:`step_state`          D_cost = 1 if A_cap_cost > A_threshold else 0                (Option 3)
"""
from __future__ import annotations

import hashlib
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence


@dataclass
class Backend:
    name: str
    url: str
    weight: float = 1.0
    pool: str = "cost"              # "cost" (cost-optimized) or "capacity" (capacity-optimized)
    cost_per_hour: float = 1.0      # C_i numerator
    max_throughput: float = 1.0     # T_i (requests / period at the breaking point)
    latency_s: float = 1.0          # L_i
    healthy: bool = True
    available: bool = True          # A_i (capacity present: GPU slot up, worker started)
    outstanding: int = 0
    ok_streak: int = 0
    fail_streak: int = 0
    served: int = 0
    errors: int = 0
    lat_ewma: Optional[float] = None
    current: float = 0.0            # smooth-WRR state

    @property
    def A(self) -> float:
        return 1.0 if (self.healthy and self.available) else 0.0

    @property
    def cost_of_inference(self) -> float:
        """README Table 1 'Cost of Inference / Second' = $/hour / breaking-point throughput."""
        return self.cost_per_hour / max(self.max_throughput, 1e-9)


def efficiency_weights(bs: Sequence[Backend]) -> List[float]:
    raw = [(b.max_throughput / (b.cost_per_hour * b.latency_s)) * b.A for b in bs]
    s = sum(raw)
    return [r / s if s > 0 else 0.0 for r in raw]


def cost_weights(bs: Sequence[Backend]) -> List[float]:
    raw = [(b.cost_per_hour / b.latency_s) for b in bs]
    s = sum(raw)
    return [r / s if s > 0 else 0.0 for r in raw]


def capacity_weights(bs: Sequence[Backend]) -> List[float]:
    s = sum(b.A for b in bs)
    return [b.A / s if s > 0 else 0.0 for b in bs]


def adjusted_throughput(max_tps: Sequence[float]) -> List[float]:
    target = sum(max_tps) / max(1, len(max_tps))
    return [min(target, t) for t in max_tps]


def step_state(avail_cost_fraction: float, threshold: float) -> int:
    """Option 3 controller: 1 = cost-optimized routing, 0 = capacity-optimized."""
    return 1 if avail_cost_fraction > threshold else 0


class Policy:
    name = "base"

    def pick(self, bs: List[Backend], key: Optional[str] = None) -> Optional[Backend]:
        raise NotImplementedError


class WeightedPolicy(Policy):
    """Smooth weighted round-robin (nginx algorithm) over available backends."""
    name = "weighted"

    def __init__(self):
        self._lock = threading.Lock()

    def pick(self, bs, key=None):
        live = [b for b in bs if b.A > 0 and b.weight > 0]
        if not live:
            return None
        with self._lock:
            total = sum(b.weight for b in live)
            for b in live:
                b.current += b.weight
            best = max(live, key=lambda b: b.current)
            best.current -= total
            return best


class RoundRobinPolicy(Policy):
    """Equal share across available backends (Option 2 / equal-routing)."""
    name = "round_robin"

    def __init__(self):
        self._i = 0
        self._lock = threading.Lock()

    def pick(self, bs, key=None):
        live = [b for b in bs if b.A > 0]
        if not live:
            return None
        with self._lock:
            self._i = (self._i + 1) % len(live)
            return live[self._i]


class LeastOutstandingPolicy(Policy):
    """Fewest in-flight requests, ties broken by EWMA latency."""
    name = "least_outstanding"

    def pick(self, bs, key=None):
        live = [b for b in bs if b.A > 0]
        if not live:
            return None
        return min(live, key=lambda b: (b.outstanding, b.lat_ewma or 0.0))


class StickyPolicy(Policy):
    """Wraps a policy with client stickiness (ALB stickiness, duration 200 s)."""

    def __init__(self, inner: Policy, ttl_s: float = 200.0):
        self.inner, self.ttl = inner, ttl_s
        self.name = f"sticky({inner.name})"
        self._map: Dict[str, tuple] = {}
        self._lock = threading.Lock()

    def pick(self, bs, key=None):
        now = time.time()
        if key:
            with self._lock:
                ent = self._map.get(key)
                if ent and now - ent[1] < self.ttl:
                    b = next((x for x in bs if x.name == ent[0] and x.A > 0), None)
                    if b is not None:
                        self._map[key] = (b.name, now)
                        return b
        b = self.inner.pick(bs, key)
        if b is not None and key:
            with self._lock:
                self._map[key] = (b.name, now)
        return b


def make_policy(name: str, sticky: bool = False) -> Policy:
    p = {"weighted": WeightedPolicy, "round_robin": RoundRobinPolicy,
         "least_outstanding": LeastOutstandingPolicy}[name]()
    return StickyPolicy(p) if sticky else p


def client_key(headers: Dict[str, str], client: Optional[str]) -> str:
    c = headers.get("cookie", "")
    for part in c.split(";"):
        if part.strip().startswith("shai_sticky="):
            return part.strip().split("=", 1)[1]
    return hashlib.sha1((client or "anon").encode()).hexdigest()[:16]
