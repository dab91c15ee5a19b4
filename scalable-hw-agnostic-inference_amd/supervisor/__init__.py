"""Single-node supervisor: GPU inventory + worker processes (replaces Karpenter
NodePools + Deployments + the device plugin).

* :class:`GPUInventory` -- the 8 GPU slots of the node (``config/node.yaml``);
  slots can be marked unavailable (fault injection / a failed GPU), which is
  what drives A_i(t) for the failover controller.
* :class:`WorkerSpec` -- one replica = (server module, GPUs, TP degree, env):
  the reference's "deployment unit" (model x accelerator x framework).
* :class:`Supervisor` -- spawns each replica as a process pinned with
  ``HIP_VISIBLE_DEVICES`` (TP groups via ``torch.distributed.run`` over RCCL),
  readiness-probes it before admitting it to the router, restarts crashed
  workers with exponential backoff (K8s restartPolicy), and exposes fault
  injection (kill a worker, fail a GPU, inject latency).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..utils.logging import get_logger

_log = get_logger("supervisor")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class WorkerSpec:
    name: str
    module: str                      # e.g. "shai_amd.serving.sd"
    gpus: List[int] = field(default_factory=list)
    tp: int = 1
    port: int = 0
    env: Dict[str, str] = field(default_factory=dict)
    pool: str = "cost"
    cost_per_hour: float = 1.0
    max_throughput: float = 1.0
    latency_s: float = 1.0
    restart: bool = True
    model_key: str = ""              # autoscaler grouping


class GPUInventory:
    def __init__(self, gpus: Optional[List[int]] = None):
        if gpus is None:
            n = int(os.environ.get("SHAI_NUM_GPUS", "0")) or _count_gpus()
            gpus = list(range(n))
        self.gpus = list(gpus)
        self.owner: Dict[int, Optional[str]] = {g: None for g in self.gpus}
        self.failed: set = set()
        self._lock = threading.Lock()

    @staticmethod
    def from_yaml(path: str) -> "GPUInventory":
        import yaml
        with open(path) as f:
            d = yaml.safe_load(f) or {}
        return GPUInventory(list(d.get("gpus", range(int(d.get("num_gpus", 8))))))

    def allocate(self, n: int, owner: str) -> Optional[List[int]]:
        with self._lock:
            free = [g for g in self.gpus if self.owner[g] is None and g not in self.failed]
            if len(free) < n:
                return None
            got = free[:n]
            for g in got:
                self.owner[g] = owner
            return got

    def release(self, owner: str):
        with self._lock:
            for g, o in self.owner.items():
                if o == owner:
                    self.owner[g] = None

    def fail(self, gpu: int):
        with self._lock:
            self.failed.add(gpu)

    def recover(self, gpu: int):
        with self._lock:
            self.failed.discard(gpu)

    @property
    def num_free(self) -> int:
        return sum(1 for g in self.gpus if self.owner[g] is None and g not in self.failed)


def _count_gpus() -> int:
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise the GPU on this image
    except Exception:
        return 0


class Supervisor:
    def __init__(self, router=None, inventory: Optional[GPUInventory] = None, log_dir: Optional[str] = None,
                 ready_timeout_s: float = 900.0):
        self.router = router
        self.inv = inventory or GPUInventory()
        self.procs: Dict[str, subprocess.Popen] = {}
        self.specs: Dict[str, WorkerSpec] = {}
        self.restarts: Dict[str, int] = {}
        self.next_restart: Dict[str, float] = {}
        self.log_dir = log_dir or os.path.join(ROOT, "gpurun_out", "workers")
        self.ready_timeout = ready_timeout_s
        self.events: List[tuple] = []
        self._stop = threading.Event()
        self._lock = threading.RLock()

    def log(self, kind, detail):
        self.events.append((time.time(), kind, detail))
        _log.info(kind, extra={"event": kind, "detail": str(detail)})

    # ------------------------------------------------------------------ lifecycle
    def _cmd(self, spec: WorkerSpec) -> List[str]:
        if spec.tp > 1:
            return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={spec.tp}",
                    "--master-addr", "127.0.0.1", f"--master-port={free_port()}", "-m", spec.module]
        return [sys.executable, "-m", spec.module]

    def start(self, spec: WorkerSpec, gpus: Optional[List[int]] = None) -> bool:
        with self._lock:
            need = max(spec.tp, len(spec.gpus) or 0, 1 if spec.env.get("DEVICE", "") != "cpu" else 0)
            if gpus is None and need:
                gpus = self.inv.allocate(need, spec.name) if not spec.gpus else spec.gpus
                if gpus is None:
                    self.log("no_capacity", spec.name)
                    return False
            spec.gpus = list(gpus or [])
            spec.port = spec.port or free_port()
            env = dict(os.environ)
            env.update({k: str(v) for k, v in spec.env.items()})
            env["PORT"] = str(spec.port)
            env["HOST"] = "127.0.0.1"
            env.setdefault("POD_NAME", spec.name)
            env.setdefault("SHAI_LOG_FORMAT", "json")   # one JSON object per line in <log_dir>/<name>.log
            if spec.tp > 1:   # every rank of the group agrees on the TP degree (serving/tp.py)
                env["TENSOR_PARALLEL_SIZE"] = str(spec.tp)
            env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
            if spec.gpus:
                env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in spec.gpus)
            os.makedirs(self.log_dir, exist_ok=True)
            out = open(os.path.join(self.log_dir, f"{spec.name}.log"), "ab")
            p = subprocess.Popen(self._cmd(spec), env=env, stdout=out, stderr=subprocess.STDOUT, cwd=ROOT,
                                 start_new_session=True)
            self.procs[spec.name] = p
            self.specs[spec.name] = spec
            self.log("start", f"{spec.name} pid={p.pid} gpus={spec.gpus} port={spec.port}")
            if self.router is not None:
                from ..router.policies import Backend
                self.router.add(Backend(spec.name, f"http://127.0.0.1:{spec.port}", pool=spec.pool,
                                        cost_per_hour=spec.cost_per_hour, max_throughput=spec.max_throughput,
                                        latency_s=spec.latency_s, healthy=False, available=False))
            return True

    def wait_ready(self, name: str, timeout: Optional[float] = None) -> bool:
        import httpx
        spec = self.specs[name]
        deadline = time.time() + (timeout or self.ready_timeout)
        while time.time() < deadline:
            p = self.procs.get(name)
            if p is None or p.poll() is not None:
                return False
            try:
                r = httpx.get(f"http://127.0.0.1:{spec.port}/readiness", timeout=2.0)
                if r.status_code == 200:
                    self._mark(name, True)
                    return True
            except Exception:
                pass
            time.sleep(0.25)
        return False

    def _mark(self, name: str, up: bool):
        if self.router is not None:
            b = self.router.get(name)
            if b is not None:
                b.available = up
                b.healthy = up
                b.fail_streak = 0
                b.ok_streak = self.router.healthy_threshold if up else 0

    def stop(self, name: str, release: bool = True):
        with self._lock:
            p = self.procs.pop(name, None)
            if p is not None and p.poll() is None:
                try:
                    os.killpg(p.pid, 15)
                except ProcessLookupError:
                    pass
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, 9)
            spec = self.specs.pop(name, None) if release else self.specs.get(name)
            if release:
                self.inv.release(name)
                if self.router is not None:
                    self.router.remove(name)
            self.log("stop", name)

    def stop_all(self):
        for n in list(self.procs):
            self.stop(n)

    # ------------------------------------------------------------------ monitoring
    def poll(self):
        """Detect exits; restart with exponential backoff; keep router availability in sync."""
        now = time.time()
        with self._lock:
            for name, p in list(self.procs.items()):
                if p.poll() is None:
                    continue
                spec = self.specs.get(name)
                self._mark(name, False)
                failed_gpu = [g for g in (spec.gpus if spec else []) if g in self.inv.failed]
                if spec is None or not spec.restart or failed_gpu:
                    self.log("exit", f"{name} rc={p.returncode} (not restarted)")
                    del self.procs[name]
                    continue
                if name not in self.next_restart:
                    k = self.restarts.get(name, 0)
                    self.next_restart[name] = now + min(60.0, 2.0 ** k)
                    self.log("crash", f"{name} rc={p.returncode}; restart #{k + 1}")
                elif now >= self.next_restart[name]:
                    self.restarts[name] = self.restarts.get(name, 0) + 1
                    del self.next_restart[name]
                    del self.procs[name]
                    self.start(spec, gpus=spec.gpus)

    def monitor(self, interval_s: float = 1.0):
        def loop():
            while not self._stop.is_set():
                self.poll()
                self._stop.wait(interval_s)
        t = threading.Thread(target=loop, daemon=True, name="supervisor")
        t.start()
        return t

    def shutdown(self):
        self._stop.set()
        self.stop_all()

    # ------------------------------------------------------------------ scaling / faults
    def replicas(self, model_key: str) -> List[str]:
        return [n for n, s in self.specs.items() if s.model_key == model_key and n in self.procs]

    def kill(self, name: str, sig: int = 9):
        """Fault injection: hard-kill a worker (it will be restarted if its spec allows)."""
        p = self.procs.get(name)
        if p is not None:
            os.killpg(p.pid, sig)
            self.log("inject_kill", name)

    def rank_pids(self, name: str) -> Dict[int, int]:
        """{rank: pid} of the worker processes of a TP group (the children ``torch.distributed.run`` started,
        identified by their RANK environment variable); {} for a TP1 worker."""
        p = self.procs.get(name)
        if p is None:
            return {}
        import psutil
        out = {}
        try:
            for c in psutil.Process(p.pid).children(recursive=True):
                try:
                    r = c.environ().get("RANK")
                except (psutil.Error, OSError):
                    continue
                if r is not None:
                    out[int(r)] = c.pid
        except psutil.Error:
            pass
        return out

    def kill_rank(self, name: str, rank: int, sig: int = 9) -> bool:
        """Fault injection: hard-kill ONE rank of a TP group (by its exact PID).  The launcher then stops the
        other ranks and the group is restarted whole (if its spec allows)."""
        pid = self.rank_pids(name).get(rank)
        if pid is None:
            return False
        os.kill(pid, sig)
        self.log("inject_kill_rank", f"{name} rank={rank} pid={pid}")
        return True

    def fail_gpu(self, gpu: int):
        """Fault injection: take a GPU out of the inventory and kill the replica using it."""
        self.inv.fail(gpu)
        self.log("inject_gpu_fail", str(gpu))
        for n, s in list(self.specs.items()):
            if gpu in s.gpus and n in self.procs:
                self._mark(n, False)
                self.kill(n)
