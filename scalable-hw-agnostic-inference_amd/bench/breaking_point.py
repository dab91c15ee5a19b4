"""Breaking-point finder (find-compute-breaking-point.yaml:21-56): against ONE
replica, ramp closed-loop clients 1 -> max_clients (the reference: 1 -> 25, 5 min
per step) and report the last step before throughput plateaus or p50 latency
exceeds the SLO (README.md:125: latency > 900 ms).
"""
from __future__ import annotations

import argparse
import json
import threading
import time
from typing import List, Optional

from .client import run_clients


def find_breaking_point(url: str, max_clients: int = 25, step_s: float = 300.0, slo_p50_s: float = 0.9,
                        plateau: float = 0.03, method: str = "GET", body: Optional[dict] = None,
                        clients_seq: Optional[List[int]] = None, progress_s: float = 0.0,
                        on_step=None) -> dict:
    """``progress_s`` > 0: a heartbeat line every progress_s seconds during a hold (long 300 s holds under a
    watchdog that takes a silent process for hung); ``on_step(step_dict)`` after every completed step."""
    steps = []
    best = None
    for n in (clients_seq or range(1, max_clients + 1)):
        stop = threading.Event()
        if progress_s > 0:
            def beat(n=n, t0=time.time()):
                while not stop.wait(progress_s):
                    print(f"  hold {n} clients: {time.time() - t0:.0f} s", flush=True)
            threading.Thread(target=beat, daemon=True).start()
        try:
            res = run_clients(n, url, step_s, method=method, body=body)
        finally:
            stop.set()
        s = {"clients": n, **res.summary()}
        steps.append(s)
        if on_step is not None:
            on_step(s)
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
    ap.add_argument("--clients", default="", help="comma-separated client counts (default 1..max-clients)")
    ap.add_argument("--progress-seconds", type=float, default=60.0)
    a = ap.parse_args()
    seq = [int(c) for c in a.clients.split(",") if c] or None
    print(json.dumps(find_breaking_point(a.url, a.max_clients, a.step_seconds, a.slo_p50, clients_seq=seq,
                                         progress_s=a.progress_seconds,
                                         on_step=lambda s: print(json.dumps(s), flush=True)), indent=1))


if __name__ == "__main__":
    main()
