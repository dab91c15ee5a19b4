"""GPU + worker health monitoring for the supervisor (replaces the reference's K8s
readiness probes / ALB unhealthy threshold / Karpenter capacity signals, sd21-weighted-routing-ing.yaml:9-14,
capacity-checker-config.yaml:19-74).

* Device health: uncorrectable ECC count growth, hotspot temperature over a limit, or a device the
  management library no longer reports -> the slot is failed in the inventory (its replica is killed and
  not restarted on it), which lowers A_i(t) for the failover controller.  A slot whose faults clear for
  ``recover_after`` consecutive polls returns to the inventory.
* Worker hang watchdog: a started worker whose ``/health`` has not answered for ``hang_timeout_s`` is
  killed; :meth:`Supervisor.poll` then restarts it with backoff.

The device query runs in a short-lived child process (``python -m shai_amd.supervisor.health``) that
imports ``amdsmi``, so the supervisor process itself never opens the GPU driver (it spawns workers).
Tests inject a fake ``probe``.
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys
import threading
import time
from dataclasses import asdict, dataclass
from typing import Callable, Dict, List, Optional


@dataclass
class GPUHealth:
    gpu: int
    ok: bool = True
    reason: str = ""
    temp_c: float = math.nan
    ecc_uncorrectable: int = 0


def query_amdsmi() -> List[dict]:
    """Per-device {gpu, temp_c, ecc_uncorrectable} via amdsmi (runs in the probe child)."""
    import amdsmi
    out = []
    amdsmi.amdsmi_init()
    try:
        for i, h in enumerate(amdsmi.amdsmi_get_processor_handles()):
            rec = {"gpu": i, "temp_c": float("nan"), "ecc_uncorrectable": 0}
            try:
                rec["temp_c"] = float(amdsmi.amdsmi_get_temp_metric(
                    h, amdsmi.AmdSmiTemperatureType.HOTSPOT, amdsmi.AmdSmiTemperatureMetric.CURRENT))
            except Exception as e:  # metric not exposed by this driver: not a fault
                rec["temp_note"] = repr(e)[:120]
            try:
                rec["ecc_uncorrectable"] = int(amdsmi.amdsmi_get_gpu_total_ecc_count(h).get("uncorrectable_count", 0))
            except Exception as e:
                rec["ecc_note"] = repr(e)[:120]
            out.append(rec)
    finally:
        amdsmi.amdsmi_shut_down()
    return out


def probe_subprocess(timeout_s: float = 20.0) -> Optional[List[dict]]:
    """Device records from a child process; None when no management library / device is available."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    try:
        r = subprocess.run([sys.executable, "-m", "shai_amd.supervisor.health"], capture_output=True, text=True,
                           timeout=timeout_s, cwd=root, env=env)
        if r.returncode != 0:
            return None
        recs = json.loads(r.stdout.strip().splitlines()[-1])
        return recs if isinstance(recs, list) else None
    except Exception:
        return None


def _http_ok(url: str, timeout: float) -> bool:
    try:
        import httpx
        return httpx.get(url, timeout=timeout).status_code == 200
    except Exception:
        return False


class GPUHealthMonitor:
    def __init__(self, supervisor, probe: Callable[[], Optional[List[dict]]] = probe_subprocess,
                 max_temp_c: float = 105.0, hang_timeout_s: float = 120.0, recover_after: int = 3,
                 http_get: Callable[[str, float], bool] = _http_ok):
        self.sup = supervisor
        self.probe = probe
        self.max_temp_c = max_temp_c
        self.hang_timeout_s = hang_timeout_s
        self.recover_after = recover_after
        self.http_get = http_get
        self.baseline_ecc: Dict[int, int] = {}
        self.clean_polls: Dict[int, int] = {}
        self.last_ok: Dict[str, float] = {}
        self.state: Dict[int, GPUHealth] = {}
        self._stop = threading.Event()

    # ------------------------------------------------------------------ devices
    def check_devices(self) -> Dict[int, GPUHealth]:
        recs = self.probe()
        if recs is None:  # no management library / no GPU (CPU box): nothing to judge
            return self.state
        seen = set()
        for r in recs:
            g = int(r["gpu"])
            seen.add(g)
            h = GPUHealth(g, temp_c=float(r.get("temp_c", math.nan)),
                          ecc_uncorrectable=int(r.get("ecc_uncorrectable", 0)))
            base = self.baseline_ecc.setdefault(g, h.ecc_uncorrectable)
            if r.get("error"):
                h.ok, h.reason = False, f"query error: {r['error']}"
            elif h.ecc_uncorrectable > base:
                h.ok, h.reason = False, f"uncorrectable ECC {base} -> {h.ecc_uncorrectable}"
                self.baseline_ecc[g] = h.ecc_uncorrectable   # acted on once; only NEW errors count again
            elif not math.isnan(h.temp_c) and h.temp_c > self.max_temp_c:
                h.ok, h.reason = False, f"hotspot {h.temp_c:.0f} C > {self.max_temp_c:.0f} C"
            self._apply(h)
        for g in self.sup.inv.gpus:  # a slot the library no longer reports
            if g not in seen:
                self._apply(GPUHealth(g, ok=False, reason="device missing"))
        return self.state

    def _apply(self, h: GPUHealth):
        self.state[h.gpu] = h
        inv = self.sup.inv
        if h.gpu not in inv.gpus:
            return
        if not h.ok:
            self.clean_polls[h.gpu] = 0
            if h.gpu not in inv.failed:
                self.sup.log("gpu_fault", f"{h.gpu}: {h.reason}")
                self.sup.fail_gpu(h.gpu)
            return
        if h.gpu in inv.failed:
            n = self.clean_polls.get(h.gpu, 0) + 1
            self.clean_polls[h.gpu] = n
            if n >= self.recover_after:
                self.baseline_ecc[h.gpu] = h.ecc_uncorrectable
                inv.recover(h.gpu)
                self.sup.log("gpu_recover", str(h.gpu))

    # ------------------------------------------------------------------ workers
    def check_workers(self, now: Optional[float] = None) -> List[str]:
        """Kill workers whose /health has not answered for hang_timeout_s; returns the names killed."""
        now = time.time() if now is None else now
        killed = []
        for name, spec in list(self.sup.specs.items()):
            p = self.sup.procs.get(name)
            if p is None or p.poll() is not None or not spec.port:
                self.last_ok.pop(name, None)
                continue
            if self.http_get(f"http://127.0.0.1:{spec.port}/health", 2.0):
                self.last_ok[name] = now
                continue
            since = self.last_ok.setdefault(name, now)
            if now - since > self.hang_timeout_s:
                self.sup.log("hang", f"{name}: /health silent for {now - since:.0f}s")
                self.sup.kill(name)
                self.last_ok.pop(name, None)
                killed.append(name)
        return killed

    def run(self, interval_s: float = 10.0):
        def loop():
            while not self._stop.is_set():
                try:
                    self.check_devices()
                    self.check_workers()
                except Exception as e:  # the monitor must never take the node down
                    self.sup.log("health_error", repr(e)[:200])
                self._stop.wait(interval_s)
        t = threading.Thread(target=loop, daemon=True, name="gpu-health")
        t.start()
        return t

    def stop(self):
        self._stop.set()

    def snapshot(self) -> List[dict]:
        return [asdict(h) for h in sorted(self.state.values(), key=lambda h: h.gpu)]


if __name__ == "__main__":  # probe child: one JSON line of device records
    try:
        print(json.dumps(query_amdsmi()))
    except Exception as e:
        print(json.dumps({"unavailable": repr(e)[:200]}))
        sys.exit(2)
