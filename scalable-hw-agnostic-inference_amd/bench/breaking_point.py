"""Breaking-point finder (find-compute-breaking-point.yaml:21-56): against ONE
replica, ramp closed-loop clients 1 -> max_clients (the reference: 1 -> 25, 5 min
per step) and report the last step before throughput plateaus or p50 latency
exceeds the SLO (README.md:125: latency > 900 ms).
"""
from __future__ import annotations

import argparse
import json
from typing import List, Optional

from .client import run_clients


def find_breaking_point(url: str, max_clients: int = 25, step_s: float = 300.0, slo_p50_s: float = 0.9,
                        plateau: float = 0.03, method: str = "GET", body: Optional[dict] = None,
                        clients_seq: Optional[List[int]] = None) -> dict:
    steps = []
    best = None
    for n in (clients_seq or range(1, max_clients + 1)):
        res = run_clients(n, url, step_s, method=method, body=body)
        s = {"clients": n, **res.summary()}
        steps.append(s)
        prev = steps[-2] if len(steps) > 1 else None
        flat = prev is not None and s["throughput_rps"] <= prev["throughput_rps"] * (1 + plateau)
        if s["p50_s"] > slo_p50_s or flat:
            break
        best = s
    return {"breaking_point": best, "steps": steps,
            "throughput_per_min": round(60 * best["throughput_rps"], 2) if best else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--max-clients", type=int, default=25)
    ap.add_argument("--step-seconds", type=float, default=300.0)
    ap.add_argument("--slo-p50", type=float, default=0.9)
    a = ap.parse_args()
    print(json.dumps(find_breaking_point(a.url, a.max_clients, a.step_seconds, a.slo_p50), indent=1))


if __name__ == "__main__":
    main()
