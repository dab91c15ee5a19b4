"""Local L7 router: replaces the reference's ALB Ingress + per-unit Services.

* Reverse proxy (any method/path) to one of the registered replicas, chosen by a
  policy (:mod:`.policies`: weighted / round-robin / least-outstanding, optional
  200 s stickiness), retrying once on a different replica on connection errors.
* Active health checks with the ALB's thresholds (sd21-weighted-routing-ing.yaml:9-14):
  GET /health every 10 s, healthy after 2 successes, unhealthy after 10 failures,
  success codes 200-301.
* Per-replica in-flight counts, EWMA latency and served/error counters; the
  router's own ``/router/state`` and ``/metrics`` feed the autoscaler and the
  failover controller; ``/router/policy`` switches policy / weights at runtime
  (what capacity-checker-deploy.yaml:26-49 does with ``kubectl apply`` of
  alternative Ingress manifests).
"""
import asyncio  # no `from __future__ import annotations`: FastAPI must resolve the local Request type
import threading
import time
from typing import Dict, List, Optional

from .policies import (Backend, Policy, adjusted_throughput, capacity_weights, client_key, cost_weights,
                       efficiency_weights, make_policy, step_state)

HOP_HEADERS = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailers",
               "transfer-encoding", "upgrade", "content-length", "host"}


class Router:
    def __init__(self, backends: Optional[List[Backend]] = None, policy: str = "weighted", sticky: bool = False,
                 health_interval_s: float = 10.0, healthy_threshold: int = 2, unhealthy_threshold: int = 10,
                 timeout_s: float = 600.0):
        self.backends: List[Backend] = list(backends or [])
        self.policy_name = policy
        self.policy: Policy = make_policy(policy, sticky)
        self.health_interval = health_interval_s
        self.healthy_threshold, self.unhealthy_threshold = healthy_threshold, unhealthy_threshold
        self.timeout = timeout_s
        self._lock = threading.Lock()
        self.events: List[tuple] = []

    # ------------------------------------------------------------------ registry
    def add(self, b: Backend):
        with self._lock:
            self.backends = [x for x in self.backends if x.name != b.name] + [b]
        self.log("add", b.name)

    def remove(self, name: str):
        with self._lock:
            self.backends = [x for x in self.backends if x.name != name]
        self.log("remove", name)

    def get(self, name: str) -> Optional[Backend]:
        return next((b for b in self.backends if b.name == name), None)

    def set_policy(self, name: str, weights: Optional[Dict[str, float]] = None, sticky: bool = False):
        self.policy = make_policy(name, sticky)
        self.policy_name = name
        if weights:
            for b in self.backends:
                if b.name in weights:
                    b.weight = float(weights[b.name])
        self.log("policy", name)

    def apply_efficiency_weights(self):
        for b, w in zip(self.backends, efficiency_weights(self.backends)):
            b.weight = w

    def log(self, kind: str, detail: str):
        self.events.append((time.time(), kind, detail))
        if len(self.events) > 10000:
            self.events = self.events[-5000:]

    def pick(self, key: Optional[str] = None, exclude=()) -> Optional[Backend]:
        bs = [b for b in self.backends if b.name not in exclude]
        return self.policy.pick(bs, key)

    # ------------------------------------------------------------------ health
    def record_health(self, b: Backend, ok: bool):
        if ok:
            b.ok_streak += 1
            b.fail_streak = 0
            if not b.healthy and b.ok_streak >= self.healthy_threshold:
                b.healthy = True
                self.log("healthy", b.name)
        else:
            b.fail_streak += 1
            b.ok_streak = 0
            if b.healthy and b.fail_streak >= self.unhealthy_threshold:
                b.healthy = False
                self.log("unhealthy", b.name)

    async def check_once(self, client):
        async def one(b):
            try:
                r = await client.get(b.url.rstrip("/") + "/health", timeout=5.0)
                ok = 200 <= r.status_code <= 301
            except Exception:
                ok = False
            self.record_health(b, ok)
        await asyncio.gather(*(one(b) for b in list(self.backends)))

    async def health_loop(self):
        import httpx
        async with httpx.AsyncClient() as client:
            while True:
                await self.check_once(client)
                await asyncio.sleep(self.health_interval)

    def state(self) -> dict:
        return {"policy": self.policy_name,
                "backends": [{"name": b.name, "url": b.url, "weight": b.weight, "pool": b.pool, "healthy": b.healthy,
                              "available": b.available, "outstanding": b.outstanding, "served": b.served,
                              "errors": b.errors, "lat_ewma": b.lat_ewma} for b in self.backends]}


def create_app(router: Router, start_health: bool = True):
    import httpx
    from fastapi import FastAPI, Request, Response
    from fastapi.responses import JSONResponse, PlainTextResponse

    app = FastAPI(title="shai router")
    app.state.router = router
    state = {"client": None}

    @app.on_event("startup")
    async def _startup():
        state["client"] = httpx.AsyncClient(timeout=router.timeout)
        if start_health:
            app.state.health_task = asyncio.create_task(router.health_loop())

    @app.on_event("shutdown")
    async def _shutdown():
        if state["client"] is not None:
            await state["client"].aclose()

    @app.get("/router/state")
    def get_state():
        return router.state()

    @app.post("/router/policy")
    async def set_policy(req: Request):
        body = await req.json()
        router.set_policy(body.get("policy", router.policy_name), body.get("weights"), bool(body.get("sticky")))
        return router.state()

    @app.get("/router/metrics", response_class=PlainTextResponse)
    def metrics():
        lines = []
        for b in router.backends:
            n = b.name.replace("-", "_")
            lines += [f'shai_router_served_total{{backend="{n}"}} {b.served}',
                      f'shai_router_errors_total{{backend="{n}"}} {b.errors}',
                      f'shai_router_outstanding{{backend="{n}"}} {b.outstanding}',
                      f'shai_router_healthy{{backend="{n}"}} {int(b.healthy)}']
        return "\n".join(lines) + "\n"

    @app.api_route("/{path:path}", methods=["GET", "POST", "PUT", "DELETE", "PATCH", "OPTIONS", "HEAD"])
    async def proxy(path: str, request: Request):
        client = state["client"] or httpx.AsyncClient(timeout=router.timeout)
        body = await request.body()
        headers = {k: v for k, v in request.headers.items() if k.lower() not in HOP_HEADERS}
        key = client_key(dict(request.headers), request.client.host if request.client else None)
        tried = []
        for attempt in range(2):
            b = router.pick(key, exclude=tried)
            if b is None:
                return JSONResponse({"detail": "no healthy backend"}, status_code=503)
            tried.append(b.name)
            b.outstanding += 1
            t0 = time.time()
            try:
                url = b.url.rstrip("/") + "/" + path
                if request.url.query:
                    url += "?" + request.url.query
                r = await client.request(request.method, url, content=body, headers=headers)
            except Exception:
                b.errors += 1
                router.record_health(b, False)
                continue
            finally:
                b.outstanding -= 1
            dt = time.time() - t0
            b.served += 1
            if r.status_code >= 500:
                b.errors += 1
            b.lat_ewma = dt if b.lat_ewma is None else 0.8 * b.lat_ewma + 0.2 * dt
            out_headers = {k: v for k, v in r.headers.items() if k.lower() not in HOP_HEADERS}
            out_headers["x-shai-backend"] = b.name
            resp = Response(content=r.content, status_code=r.status_code, headers=out_headers)
            resp.set_cookie("shai_sticky", key, max_age=200)
            return resp
        return JSONResponse({"detail": "all backends failed"}, status_code=502)

    return app


__all__ = ["Router", "Backend", "create_app", "efficiency_weights", "cost_weights", "capacity_weights",
           "adjusted_throughput", "step_state"]
