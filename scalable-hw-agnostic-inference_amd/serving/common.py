"""Shared serving plumbing for every model server.

* :class:`ServerEnv` -- the reference's environment-variable "flag system"
  (APP, POD_NAME, NODEPOOL, MODEL_ID, COMPILED_MODEL_ID, DEVICE,
  NUM_OF_RUNS_INF, MAX_NEW_TOKENS, HEIGHT, WIDTH, MAX_SEQ_LEN, GUIDANCE_SCALE,
  ... SURVEY.md 2.12) with defaults, so the same deployment env works here.
  ``DEVICE`` is accepted and validated; there is a single (gfx950) backend.
* :class:`LatencyCollector` / :func:`benchmark` -- byte-compatible percentile
  rule and report string of app/run-sd.py:49-102 / app/vllm_model_api.py:61-109.
* :class:`Metrics` -- in-process registry replacing CloudWatch
  ``put_metric_data`` (same metric names ``<APP>-counter``, ``<NODEPOOL>``,
  ``<APP>-latency``), exposed at ``GET /metrics`` (Prometheus text) and read
  directly by the router / autoscaler.
* :class:`EngineWorker` -- ONE thread owns the GPU engine; HTTP handlers submit
  work and wait on futures.  Fixes the reference's unsynchronised sharing of one
  diffusers pipeline across FastAPI's threadpool (run-sd.py:137-142,184-193).
  Optional dynamic batching: compatible requests arriving within a short window
  run as one batched engine call.
"""
from __future__ import annotations

import base64
import io
import math
import os
import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..utils import liveness as _liveness

VALID_DEVICES = {"xla", "cuda", "triton", "cpu", "rocm", "hip", "gpu", ""}


@dataclass
class ServerEnv:
    app: str = "shai"
    pod_name: str = "pod"
    nodepool: str = "mi355x"
    model_id: str = ""
    compiled_model_id: str = ""
    device: str = "rocm"
    num_inference_steps: int = 50
    max_new_tokens: int = 128
    height: int = 512
    width: int = 512
    max_seq_len: int = 512
    guidance_scale: float = 3.5
    model_path: Optional[str] = None     # local checkpoint dir (safetensors); None -> random init
    config: str = ""                     # model-size override, e.g. "tiny" for tests

    @staticmethod
    def from_env(**defaults) -> "ServerEnv":
        e = os.environ
        d = ServerEnv(**defaults)

        def g(name, cur, cast=str):
            v = e.get(name)
            return cast(v) if v not in (None, "") else cur

        d.app = g("APP", d.app)
        d.pod_name = g("POD_NAME", d.pod_name)
        d.nodepool = g("NODEPOOL", d.nodepool)
        d.model_id = g("MODEL_ID", d.model_id)
        d.compiled_model_id = g("COMPILED_MODEL_ID", d.compiled_model_id or d.model_id)
        d.device = g("DEVICE", d.device)
        d.num_inference_steps = g("NUM_OF_RUNS_INF", d.num_inference_steps, int)
        d.max_new_tokens = g("MAX_NEW_TOKENS", d.max_new_tokens, int)
        d.height = g("HEIGHT", d.height, int)
        d.width = g("WIDTH", d.width, int)
        d.max_seq_len = g("MAX_SEQ_LEN", d.max_seq_len, int)
        d.guidance_scale = g("GUIDANCE_SCALE", d.guidance_scale, float)
        d.model_path = g("SHAI_MODEL_PATH", d.model_path)
        if d.model_path is None and d.model_id and os.path.isdir(d.model_id):
            d.model_path = d.model_id
        d.config = g("SHAI_MODEL_CONFIG", d.config)
        if d.device.lower() not in VALID_DEVICES:
            raise ValueError(f"DEVICE={d.device!r} not supported (single gfx950 backend; accepted: {VALID_DEVICES})")
        return d

    @property
    def torch_device(self) -> str:
        import torch
        if self.device.lower() == "cpu" or not torch.cuda.is_available():
            return "cpu"
        return f"cuda:{torch.cuda.current_device()}"


# ----------------------------------------------------------------------------- latency
class LatencyCollector:
    """Same percentile rule as the reference (nearest rank, ceil when frac > 0.5)."""

    def __init__(self):
        self.start = None
        self.latency_list: List[float] = []

    def pre_hook(self, *args):
        self.start = time.time()

    def hook(self, *args):
        self.latency_list.append(time.time() - self.start)

    def percentile(self, percent):
        lat = self.latency_list
        pos_float = len(lat) * percent / 100
        max_pos = len(lat) - 1
        pos_floor = min(math.floor(pos_float), max_pos)
        pos_ceil = min(math.ceil(pos_float), max_pos)
        lat = sorted(lat)
        return lat[pos_ceil] if pos_float - pos_floor > 0.5 else lat[pos_floor]


def latency_report(collector: LatencyCollector, test_name: str, pod_name: Optional[str] = None) -> str:
    keys = [("Latency P0", 0), ("Latency P50", 50), ("Latency P90", 90), ("Latency P95", 95), ("Latency P99", 99),
            ("Latency P100", 100)]
    report = f"RESULT FOR {test_name} on {pod_name}:" if pod_name is not None else f"RESULT FOR {test_name}:"
    for k, p in keys:
        report += f" {k}={collector.percentile(p) * 1000:.1f}"
    return report


def benchmark(n_runs: int, test_name: str, fn: Callable[[], Any], pod_name: Optional[str] = None,
              warmup: bool = False) -> str:
    if warmup:
        fn()
    lc = LatencyCollector()
    for _ in range(max(1, n_runs)):
        lc.pre_hook()
        fn()
        lc.hook()
    return latency_report(lc, test_name, pod_name)


# ----------------------------------------------------------------------------- metrics
class Metrics:
    """Counters (sum) and latency samples; names follow the reference's CloudWatch metrics."""

    def __init__(self):
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = {}
        self.latencies: Dict[str, List[float]] = {}
        self.events: List[tuple] = []  # (time, name, value) for windowed rates (autoscaler)

    def publish(self, name: str, value: float, unit: str = "Count"):
        now = time.time()
        with self._lock:
            if unit == "Seconds":
                self.latencies.setdefault(name, []).append(float(value))
                if len(self.latencies[name]) > 10000:
                    self.latencies[name] = self.latencies[name][-5000:]
            else:
                self.counters[name] = self.counters.get(name, 0.0) + float(value)
            self.events.append((now, name, float(value)))
            if len(self.events) > 100000:
                self.events = self.events[-50000:]

    def request_done(self, env: ServerEnv, seconds: float):
        self.publish(env.app + "-counter", 1, "Count")
        self.publish(env.nodepool, 1, "Count")
        self.publish(env.app + "-latency", seconds, "Seconds")

    def rate(self, name: str, window_s: float = 60.0) -> float:
        cut = time.time() - window_s
        with self._lock:
            return sum(v for t, n, v in self.events if n == name and t >= cut)

    def render_prometheus(self) -> str:
        def clean(n):
            return "".join(ch if ch.isalnum() else "_" for ch in n)

        lines = []
        with self._lock:
            for n, v in sorted(self.counters.items()):
                lines.append(f"# TYPE {clean(n)}_total counter")
                lines.append(f"{clean(n)}_total {v}")
            for n, vals in sorted(self.latencies.items()):
                s = sorted(vals)
                lines.append(f"# TYPE {clean(n)}_seconds summary")
                for q in (0.5, 0.9, 0.99):
                    lines.append(f'{clean(n)}_seconds{{quantile="{q}"}} {s[min(len(s) - 1, int(q * len(s)))]}')
                lines.append(f"{clean(n)}_seconds_count {len(s)}")
                lines.append(f"{clean(n)}_seconds_sum {sum(s)}")
        return "\n".join(lines) + "\n"


METRICS = Metrics()


# ----------------------------------------------------------------------------- engine worker
@dataclass
class _Job:
    fn: Callable
    args: tuple
    fut: Future
    key: Any = None
    t: float = field(default_factory=time.time)


class EngineWorker:
    """Single GPU-owning thread.  ``submit(fn, *args)`` runs fn(*args) serially.

    With ``batch_fn`` set, :meth:`submit_batched` groups requests sharing
    ``key`` (e.g. same step count) arriving within ``max_wait_ms`` into one
    ``batch_fn(key, [args...]) -> [results...]`` call (up to ``max_batch``)."""

    def __init__(self, name: str = "engine", batch_fn: Optional[Callable] = None, max_batch: int = 8,
                 max_wait_ms: float = 5.0):
        self.q: "queue.Queue[_Job]" = queue.Queue()
        self.batch_fn, self.max_batch, self.max_wait = batch_fn, max_batch, max_wait_ms / 1000.0
        self.busy = 0
        self.live = _liveness.register(_liveness.Liveness())
        self.t = threading.Thread(target=self._loop, name=name, daemon=True)
        self.t.start()

    def submit(self, fn: Callable, *args) -> Future:
        f: Future = Future()
        self.live.work_pending()
        self.q.put(_Job(fn, args, f))
        return f

    def submit_batched(self, key, *args) -> Future:
        f: Future = Future()
        self.live.work_pending()
        self.q.put(_Job(None, args, f, key))
        return f

    def call(self, fn: Callable, *args, timeout: Optional[float] = None):
        return self.submit(fn, *args).result(timeout)

    @property
    def queue_depth(self) -> int:
        return self.q.qsize() + self.busy

    def _loop(self):
        import torch
        pending: List[_Job] = []
        while True:
            job = pending.pop(0) if pending else self.q.get()
            self.busy = 1
            try:
                if job.fn is not None:
                    with torch.inference_mode():
                        job.fut.set_result(job.fn(*job.args))
                    continue
                batch = [job]
                deadline = time.time() + self.max_wait
                while len(batch) < self.max_batch:
                    try:
                        nxt = self.q.get(timeout=max(0.0, deadline - time.time()))
                    except queue.Empty:
                        break
                    if nxt.fn is None and nxt.key == job.key:
                        batch.append(nxt)
                    else:
                        pending.append(nxt)
                with torch.inference_mode():
                    res = self.batch_fn(job.key, [b.args for b in batch])
                for b, r in zip(batch, res):
                    b.fut.set_result(r)
            except BaseException as e:  # propagate to callers
                if job.fn is None and "batch" in locals():
                    for b in batch:
                        if not b.fut.done():
                            b.fut.set_exception(e)
                elif not job.fut.done():
                    job.fut.set_exception(e)
            finally:
                self.busy = 0
                self.live.progress(still_pending=bool(pending) or not self.q.empty())


# ----------------------------------------------------------------------------- app factory
def png_b64(img_u8, thumbnail: Optional[int] = None) -> str:
    """uint8 HWC tensor / ndarray -> base64 PNG (optionally thumbnailed, LANCZOS)."""
    import numpy as np
    from PIL import Image
    arr = img_u8.numpy() if hasattr(img_u8, "numpy") else np.asarray(img_u8)
    im = Image.fromarray(np.ascontiguousarray(arr))
    if thumbnail:
        im.thumbnail((thumbnail, thumbnail), Image.LANCZOS)
    buf = io.BytesIO()
    im.save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode("utf-8")


def b64text(s: str) -> str:
    return base64.b64encode(s.encode()).decode()


def base_app(env: ServerEnv, title: str, spaced: bool, cors: bool = False):
    """FastAPI app with /health, /readiness, /metrics.

    ``spaced``: the *_model_api.py servers answer "<pod> is healthy"; the
    run-*.py servers concatenate without a space ("<pod>is healthy").
    """
    from fastapi import FastAPI
    from fastapi.responses import PlainTextResponse
    app = FastAPI(title=title)
    sep = " " if spaced else ""
    app.state.env = env
    app.state.ready = True

    @app.get("/health")
    def healthy():
        # liveness, not just "the HTTP server answers": 503 once an engine has had work pending without
        # progress for longer than its hang timeout (utils/liveness.py), so the router drains this replica
        # and the supervisor's watchdog restarts it
        why = _liveness.broken()
        if why is not None:
            from fastapi import HTTPException
            raise HTTPException(status_code=503, detail=f"replica broken: {why}")
        live = _liveness.worst()
        if live is not None and not live.healthy:
            from fastapi import HTTPException
            raise HTTPException(status_code=503, detail=f"engine stalled: {live.snapshot()}")
        return {"message": f"{env.pod_name}{sep}is healthy"}

    @app.get("/readiness")
    def ready():
        from fastapi import HTTPException
        if not app.state.ready:
            raise HTTPException(status_code=503, detail="warming up")
        return {"message": f"{env.pod_name}{sep}is ready"}

    @app.get("/metrics", response_class=PlainTextResponse)
    def metrics():
        return METRICS.render_prometheus()

    if cors:
        from fastapi.middleware.cors import CORSMiddleware
        app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                           allow_headers=["*"])
    return app


def mount_ui(app, title: str, endpoint: str, body_template: str, output: str = "text"):
    """Minimal /serve page (Gradio is not installed in this image): a form that
    POSTs JSON to ``endpoint`` and renders the response (text or base64 image)."""
    from fastapi.responses import HTMLResponse
    page = f"""<!doctype html><html><head><title>{title}</title></head><body>
<h3>{title}</h3><textarea id="p" rows="3" cols="80">a photo of an astronaut riding a horse on mars</textarea><br>
<button onclick="go()">Submit</button><pre id="t"></pre><img id="i"/>
<script>
async function go() {{
  const p = document.getElementById('p').value;
  const body = {body_template};
  const r = await fetch('{endpoint}', {{method: 'POST', headers: {{'Content-Type': 'application/json'}},
                                     body: JSON.stringify(body)}});
  const j = await r.json();
  const img = j.response && '{output}' === 'image' ? j.response : (j.image && '{output}' === 'image' ? j.image : null);
  if (img) document.getElementById('i').src = 'data:image/png;base64,' + img;
  document.getElementById('t').textContent = JSON.stringify(j, (k, v) =>
      (typeof v === 'string' && v.length > 200) ? v.slice(0, 200) + '...' : v, 2);
}}
</script></body></html>"""

    @app.get("/serve", response_class=HTMLResponse)
    def serve():
        return page

    return app


def run(app, port: Optional[int] = None):
    import uvicorn
    uvicorn.run(app, host=os.environ.get("HOST", "0.0.0.0"), port=int(port or os.environ.get("PORT", "8000")))
