"""Closed-loop HTTP load client (replaces app/call-model.sh: an infinite
``curl $SERVE_ENDPOINT/load/$NUM_OF_ITERATIONS/infer/$NUM_OF_INF; sleep``).

``run_clients(n, ...)`` runs n concurrent closed-loop clients for a duration
and returns per-request latencies / status codes, throughput and percentiles
(the reference's LatencyCollector rule).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

from ..serving.common import LatencyCollector


@dataclass
class LoadResult:
    latencies: List[float] = field(default_factory=list)
    codes: List[int] = field(default_factory=list)
    duration_s: float = 0.0

    @property
    def ok(self) -> int:
        return sum(1 for c in self.codes if 200 <= c < 300)

    @property
    def throughput(self) -> float:
        return self.ok / self.duration_s if self.duration_s else 0.0

    def pct(self, p) -> float:
        if not self.latencies:
            return float("nan")
        lc = LatencyCollector()
        lc.latency_list = list(self.latencies)
        return lc.percentile(p)

    def summary(self) -> dict:
        return {"requests": len(self.codes), "ok": self.ok, "errors_5xx": sum(1 for c in self.codes if c >= 500),
                "throughput_rps": round(self.throughput, 3), "p50_s": round(self.pct(50), 4),
                "p90_s": round(self.pct(90), 4), "p99_s": round(self.pct(99), 4)}


async def _client(url, method, body, stop_at, res: LoadResult, sleep_s, client):
    while time.time() < stop_at:
        t0 = time.time()
        try:
            r = await (client.post(url, json=body) if method == "POST" else client.get(url))
            code = r.status_code
        except Exception:
            code = 599
        res.latencies.append(time.time() - t0)
        res.codes.append(code)
        if sleep_s:
            await asyncio.sleep(sleep_s)


async def run_clients_async(n: int, url: str, duration_s: float, method: str = "GET", body: Optional[dict] = None,
                            sleep_s: float = 0.0, timeout_s: float = 600.0) -> LoadResult:
    import httpx
    res = LoadResult()
    t0 = time.time()
    async with httpx.AsyncClient(timeout=timeout_s) as client:
        await asyncio.gather(*(_client(url, method, body, t0 + duration_s, res, sleep_s, client) for _ in range(n)))
    res.duration_s = time.time() - t0
    return res


def run_clients(n: int, url: str, duration_s: float, **kw) -> LoadResult:
    return asyncio.run(run_clients_async(n, url, duration_s, **kw))


async def run_open_loop_async(rate_rps: float, url: str, duration_s: float, method: str = "GET",
                              body: Optional[dict] = None, seed: int = 0, timeout_s: float = 600.0) -> LoadResult:
    """Open-loop load: requests arrive as a Poisson process of ``rate_rps`` for ``duration_s`` seconds whether or
    not earlier ones have finished (real user traffic, unlike the closed-loop clients whose arrivals align with
    the server's completions); every request's latency is recorded."""
    import random

    import httpx
    res = LoadResult()
    rng = random.Random(seed)
    t0 = time.time()

    async def one(client):
        s = time.time()
        try:
            r = await (client.post(url, json=body) if method == "POST" else client.get(url))
            code = r.status_code
        except Exception:
            code = 599
        res.latencies.append(time.time() - s)
        res.codes.append(code)
    async with httpx.AsyncClient(timeout=timeout_s, limits=httpx.Limits(max_connections=1000)) as client:
        tasks, t = [], t0
        while True:
            t += rng.expovariate(rate_rps)
            if t >= t0 + duration_s:
                break
            await asyncio.sleep(max(0.0, t - time.time()))
            tasks.append(asyncio.create_task(one(client)))
        await asyncio.gather(*tasks)
    res.duration_s = time.time() - t0
    return res


def run_open_loop(rate_rps: float, url: str, duration_s: float, **kw) -> LoadResult:
    return asyncio.run(run_open_loop_async(rate_rps, url, duration_s, **kw))


def main():
    ap = argparse.ArgumentParser(description="closed-loop load client (call-model.sh equivalent)")
    ap.add_argument("--endpoint", default=os.environ.get("SERVE_ENDPOINT", "http://127.0.0.1:8000"))
    ap.add_argument("--iterations", type=int, default=int(os.environ.get("NUM_OF_ITERATIONS", "1")))
    ap.add_argument("--inf", type=int, default=int(os.environ.get("NUM_OF_INF", "10")))
    ap.add_argument("--sleep", type=float, default=float(os.environ.get("SLEEP_TIME", "0")))
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--duration", type=float, default=60.0)
    a = ap.parse_args()
    url = f"{a.endpoint.rstrip('/')}/load/{a.iterations}/infer/{a.inf}"
    print(json.dumps(run_clients(a.clients, url, a.duration, sleep_s=a.sleep).summary()))


if __name__ == "__main__":
    main()
