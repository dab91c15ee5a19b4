"""Load shapes driving the number of concurrent clients over time.

* ``sine``   -- app/appsimulator.sh:26-57: clients = int(sin(i)*40)*CLIENT_SCALE_RATIO + MIN_AT_CYCLE_START,
               i advancing by RADIAN_INTERVAL up to RADIAN_MAX (negative counts clamp to the minimum).
* ``cosine`` -- load-cosine-simu.yaml:28-69: MIN + (MAG-MIN) * (1 + cos(2*pi*t/PERIOD)) / 2, MAG=100, PERIOD=900.
The phase is persisted to a JSON state file (the reference keeps it in SQS).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time
from typing import Iterator, Tuple


def sine_clients(i: float, scale: float = 1.0, minimum: int = 1) -> int:
    return max(minimum, int(math.sin(i) * 40) * int(scale) + minimum)


def cosine_clients(t: float, minimum: int = 1, magnitude: int = 100, period: float = 900.0) -> int:
    return int(minimum + (magnitude - minimum) * (1 + math.cos(2 * math.pi * t / period)) / 2)


def schedule(shape: str, steps: int, step_s: float, **kw) -> Iterator[Tuple[float, int]]:
    for k in range(steps):
        if shape == "sine":
            i = kw.get("radian_interval", 0.1) * k % kw.get("radian_max", 3.14)
            yield k * step_s, sine_clients(i, kw.get("scale", 1.0), kw.get("minimum", 1))
        else:
            yield k * step_s, cosine_clients(k * step_s, kw.get("minimum", 1), kw.get("magnitude", 100),
                                             kw.get("period", 900.0))


def drive(shape: str, url: str, steps: int, step_s: float, state_file: str = "", **kw):
    """Run the shape against ``url`` (closed-loop clients per step); returns per-step summaries."""
    from .client import run_clients
    start = 0
    if state_file and os.path.exists(state_file):
        start = json.load(open(state_file)).get("step", 0)
    out = []
    for k, (t, n) in enumerate(schedule(shape, steps + start, step_s, **kw)):
        if k < start:
            continue
        res = run_clients(n, url, step_s)
        out.append({"t": t, "clients": n, **res.summary()})
        if state_file:
            json.dump({"step": k + 1}, open(state_file, "w"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", choices=["sine", "cosine"], default="cosine")
    ap.add_argument("--url", default=os.environ.get("SERVE_ENDPOINT", "http://127.0.0.1:8000") + "/load/1/infer/10")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--step-seconds", type=float, default=60.0)
    ap.add_argument("--state-file", default="")
    ap.add_argument("--minimum", type=int, default=int(os.environ.get("MIN_AT_CYCLE_START", "1")))
    ap.add_argument("--scale", type=float, default=float(os.environ.get("CLIENT_SCALE_RATIO", "1")))
    ap.add_argument("--magnitude", type=int, default=100)
    ap.add_argument("--period", type=float, default=900.0)
    a = ap.parse_args()
    for row in drive(a.shape, a.url, a.steps, a.step_seconds, a.state_file, minimum=a.minimum, scale=a.scale,
                     magnitude=a.magnitude, period=a.period):
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
