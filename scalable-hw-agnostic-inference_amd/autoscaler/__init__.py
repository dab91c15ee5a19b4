"""Target-throughput autoscaler (replaces KEDA ScaledObjects on CloudWatch,
sd21-scaledobject*.yaml): desired = ceil(SUM(<app>-counter over the window) /
targetMetricValue), clamped to [min, max] and to free GPU slots; scale-up is
immediate, scale-down waits for a stabilisation window (HPA behaviour).
Per-replica targets can come from the README's adjusted-throughput rule
(``router.policies.adjusted_throughput``).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Callable, List, Optional


@dataclass
class ScaleTarget:
    model_key: str
    target_per_replica: float          # KEDA targetMetricValue (requests per window)
    min_replicas: int = 1
    max_replicas: int = 8
    window_s: float = 60.0
    scale_down_stabilization_s: float = 300.0


class Autoscaler:
    def __init__(self, supervisor, make_spec: Callable[[str, int], object], metric: Callable[[str, float], float]):
        """make_spec(model_key, index) -> WorkerSpec; metric(model_key, window_s) -> request count."""
        self.sup = supervisor
        self.make_spec = make_spec
        self.metric = metric
        self.targets: List[ScaleTarget] = []
        self._below_since = {}
        self.decisions: List[tuple] = []

    def add(self, t: ScaleTarget):
        self.targets.append(t)

    def desired(self, t: ScaleTarget, value: float) -> int:
        d = math.ceil(value / max(t.target_per_replica, 1e-9)) if value > 0 else t.min_replicas
        return max(t.min_replicas, min(t.max_replicas, d))

    def tick(self, now: Optional[float] = None):
        now = now or time.time()
        for t in self.targets:
            cur = self.sup.replicas(t.model_key)
            want = self.desired(t, self.metric(t.model_key, t.window_s))
            if want > len(cur):
                self._below_since.pop(t.model_key, None)
                for i in range(want - len(cur)):
                    spec = self.make_spec(t.model_key, len(cur) + i)
                    if not self.sup.start(spec):
                        break
                self.decisions.append((now, t.model_key, len(cur), want))
            elif want < len(cur):
                since = self._below_since.setdefault(t.model_key, now)
                if now - since >= t.scale_down_stabilization_s:
                    for name in sorted(cur)[want:]:
                        self.sup.stop(name)
                    self._below_since.pop(t.model_key, None)
                    self.decisions.append((now, t.model_key, len(cur), want))
            else:
                self._below_since.pop(t.model_key, None)


def router_rate_metric(router, prefix_by_model=None):
    """Request count per model over a window from the router's served counters."""
    hist = {}

    def metric(model_key: str, window_s: float) -> float:
        now = time.time()
        total = sum(b.served for b in router.backends if (prefix_by_model or {}).get(model_key, model_key) in b.name)
        h = hist.setdefault(model_key, [])
        h.append((now, total))
        while h and now - h[0][0] > window_s:
            h.pop(0)
        return float(total - h[0][1]) if h else 0.0

    return metric
