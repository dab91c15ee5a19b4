"""Node launcher: one 8x MI355X node = supervisor + router + autoscaler +
failover controller, configured by a YAML file (config/node.yaml) -- the local
equivalent of the reference's NodePools + Deployments + Services/Ingress +
ScaledObjects + capacity checker.

  python -m shai_amd.launch --config config/node.yaml
"""
import argparse
import time

from .autoscaler import Autoscaler, ScaleTarget, router_rate_metric
from .controller.failover import FailoverController
from .router import Router, create_app
from .serving.common import run
from .supervisor import GPUInventory, Supervisor, WorkerSpec
from .supervisor.health import GPUHealthMonitor
from .utils.config import load_node_config


def spec_factory(dep: dict):
    def make(model_key: str, idx: int) -> WorkerSpec:
        return WorkerSpec(name=f"{dep['name']}-{idx}", module=dep["module"], tp=int(dep.get("tp", 1)),
                          env={k: str(v) for k, v in (dep.get("env") or {}).items()}, pool=dep.get("pool", "cost"),
                          cost_per_hour=float(dep.get("cost_per_hour", 1.0)),
                          max_throughput=float(dep.get("max_throughput", 1.0)),
                          latency_s=float(dep.get("latency_s", 1.0)), model_key=dep["name"])
    return make


def build(cfg: dict):
    inv = GPUInventory(cfg.get("gpus"))
    rcfg = cfg.get("router", {})
    router = Router(policy=rcfg.get("policy", "weighted"), sticky=bool(rcfg.get("sticky", False)),
                    health_interval_s=float(rcfg.get("health_interval_s", 10)))
    sup = Supervisor(router, inv)
    makers = {d["name"]: spec_factory(d) for d in cfg.get("deployments", [])}
    scaler = Autoscaler(sup, lambda key, i: makers[key](key, i), router_rate_metric(router))
    for d in cfg.get("deployments", []):
        for i in range(int(d.get("replicas", 1))):
            sup.start(makers[d["name"]](d["name"], i))
        a = d.get("autoscale")
        if a:
            scaler.add(ScaleTarget(d["name"], float(a["target_per_replica"]), int(a.get("min", 1)),
                                   int(a.get("max", len(inv.gpus))), float(a.get("window_s", 60)),
                                   float(a.get("scale_down_stabilization_s", 300))))
    fo = FailoverController(router, float(cfg.get("failover", {}).get("threshold", 0.5)),
                            float(cfg.get("failover", {}).get("fallback_hold_s", 60)))
    return router, sup, scaler, fo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config/node.yaml")
    a = ap.parse_args()
    cfg = load_node_config(a.config).as_dict()   # validated (utils/config.py), SHAI_NODE__* env overrides
    router, sup, scaler, fo = build(cfg)
    for name in list(sup.specs):
        sup.wait_ready(name)
    router.apply_efficiency_weights()
    sup.monitor()
    hc = cfg.get("health", {})
    GPUHealthMonitor(sup, max_temp_c=float(hc.get("max_temp_c", 105)),
                     hang_timeout_s=float(hc.get("hang_timeout_s", 120))).run(float(hc.get("interval_s", 10)))
    fo.run(float(cfg.get("failover", {}).get("interval_s", 300)))

    import threading

    def scale_loop():
        while True:
            scaler.tick()
            time.sleep(float(cfg.get("autoscale_interval_s", 30)))
    threading.Thread(target=scale_loop, daemon=True).start()
    try:
        run(create_app(router), port=int(cfg.get("router", {}).get("port", 8080)))
    finally:
        sup.shutdown()


if __name__ == "__main__":
    main()
