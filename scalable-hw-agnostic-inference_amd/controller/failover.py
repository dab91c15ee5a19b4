"""Capacity failover / fallback controller (README Option 3; replaces
capacity-checker-config.yaml + capacity-checker-deploy.yaml:26-49, which polls
CloudWatch Logs for Karpenter "insufficient capacity" every 300 s and
kubectl-applies the equal-routing or weighted-routing manifests).

State D_cost(t) = step(A_cost(t) > A_threshold) where A_cost is the fraction of
cost-optimized replicas that are available (GPU slot healthy, worker ready,
router health checks passing).
* cost -> capacity (failover): when A_cost <= threshold, route round-robin over
  every available replica (capacity-optimized, Option 2).
* capacity -> cost (fallback): when A_cost recovers above the threshold and the
  condition holds for ``fallback_hold_s`` (or a new load wave starts, as the
  reference detects via the load deployment's ready replicas in [1, 5]),
  restore the weighted cost-optimized distribution (Option 1 / eq. 1 weights).
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Dict, List, Optional

from ..router.policies import efficiency_weights, step_state


class FailoverController:
    def __init__(self, router, threshold: float = 0.5, fallback_hold_s: float = 60.0,
                 cost_weights: Optional[Dict[str, float]] = None,
                 new_wave: Optional[Callable[[], bool]] = None):
        self.router = router
        self.threshold = threshold
        self.fallback_hold_s = fallback_hold_s
        self.cost_weights = cost_weights
        self.new_wave = new_wave
        self.mode = "cost"
        self._ok_since: Optional[float] = None
        self.transitions: List[tuple] = []
        self._stop = threading.Event()

    def a_cost(self) -> float:
        pool = [b for b in self.router.backends if b.pool == "cost"]
        if not pool:
            return 1.0
        return sum(b.A for b in pool) / len(pool)

    def _weights(self) -> Dict[str, float]:
        if self.cost_weights:
            return dict(self.cost_weights)
        bs = self.router.backends
        return {b.name: w for b, w in zip(bs, efficiency_weights(bs))}

    def evaluate(self, now: Optional[float] = None) -> str:
        now = now or time.time()
        a = self.a_cost()
        d_cost = step_state(a, self.threshold)
        if self.mode == "cost" and d_cost == 0:
            self.router.set_policy("round_robin")
            self.mode = "capacity"
            self._ok_since = None
            self.transitions.append((now, "failover", a))
        elif self.mode == "capacity":
            if d_cost == 1:
                self._ok_since = self._ok_since or now
                wave = self.new_wave() if self.new_wave else False
                if wave or now - self._ok_since >= self.fallback_hold_s:
                    self.router.set_policy("weighted", self._weights())
                    self.mode = "cost"
                    self.transitions.append((now, "fallback", a))
            else:
                self._ok_since = None
        return self.mode

    def run(self, interval_s: float = 300.0):
        def loop():
            while not self._stop.is_set():
                self.evaluate()
                self._stop.wait(interval_s)
        t = threading.Thread(target=loop, daemon=True, name="failover")
        t.start()
        return t

    def stop(self):
        self._stop.set()
