"""Router / supervisor / autoscaler / failover / load-generator tests on CPU with
model-free fake workers (real processes, real HTTP)."""
import math
import os
import threading
import time
from collections import Counter

import pytest

from shai_amd.router import Router, create_app
from shai_amd.router.policies import (Backend, StickyPolicy, WeightedPolicy, adjusted_throughput, capacity_weights,
                                      cost_weights, efficiency_weights, step_state)

README_UNITS = [  # README.md Table 1 / 2: (name, $/h, breaking-point throughput, latency s)
    ("sd21-inf2", 0.7582, 105, 0.67), ("sd21-trn1", 1.3438, 130, 0.51), ("sd21-g5-triton", 1.0060, 90, 0.68),
    ("sd21-g6-triton", 0.8048, 61, 0.96), ("sd21-g5-cuda", 1.0060, 60, 0.92)]


def units():
    return [Backend(n, f"http://x/{n}", cost_per_hour=c, max_throughput=t, latency_s=l) for n, c, t, l in README_UNITS]


def test_readme_formulas():
    bs = units()
    w = efficiency_weights(bs)
    assert abs(sum(w) - 1) < 1e-9 and max(range(5), key=lambda i: w[i]) == 0  # inf2: T/(C L) = 206.7
    assert [round(b.cost_of_inference, 5) for b in bs][:1] == [round(0.7582 / 105, 5)]
    assert adjusted_throughput([105, 130, 90, 61, 60]) == [89.2, 89.2, 89.2, 61, 60]  # README Table 2
    bs[0].available = False
    assert capacity_weights(bs)[0] == 0 and abs(sum(capacity_weights(bs)) - 1) < 1e-9
    assert abs(sum(cost_weights(bs)) - 1) < 1e-9
    assert step_state(0.6, 0.5) == 1 and step_state(0.5, 0.5) == 0


def test_weighted_and_sticky_policies():
    bs = [Backend("a", "u", weight=40), Backend("b", "u", weight=20), Backend("c", "u", weight=40)]
    p = WeightedPolicy()
    cnt = Counter(p.pick(bs).name for _ in range(1000))
    assert cnt == Counter({"a": 400, "b": 200, "c": 400})  # smooth WRR is exact over a full cycle
    s = StickyPolicy(WeightedPolicy())
    first = s.pick(bs, "client1").name
    assert all(s.pick(bs, "client1").name == first for _ in range(20))
    bs[[b.name for b in bs].index(first)].healthy = False
    assert s.pick(bs, "client1").name != first


def test_health_thresholds():
    r = Router([Backend("a", "u")], healthy_threshold=2, unhealthy_threshold=10)
    b = r.backends[0]
    for _ in range(9):
        r.record_health(b, False)
    assert b.healthy
    r.record_health(b, False)
    assert not b.healthy
    r.record_health(b, True)
    assert not b.healthy
    r.record_health(b, True)
    assert b.healthy


@pytest.fixture
def fake_fleet(tmp_path):
    from shai_amd.supervisor import GPUInventory, Supervisor, WorkerSpec
    router = Router(policy="weighted", health_interval_s=0.2, unhealthy_threshold=1, healthy_threshold=1)
    sup = Supervisor(router, GPUInventory([0, 1, 2]), log_dir=str(tmp_path))
    specs = [WorkerSpec(f"w{i}", "shai_amd.supervisor.fake_worker", env={"DEVICE": "cpu", "FAKE_LATENCY_S": "0.01"},
                        pool="cost" if i < 2 else "capacity", model_key="fake") for i in range(3)]
    for s in specs:
        assert sup.start(s)
    for s in specs:
        assert sup.wait_ready(s.name, timeout=120), open(os.path.join(tmp_path, f"{s.name}.log")).read()[-2000:]
    yield router, sup
    sup.shutdown()


def test_router_supervisor_end_to_end(fake_fleet):
    from fastapi.testclient import TestClient
    router, sup = fake_fleet
    router.set_policy("weighted", {"w0": 2, "w1": 1, "w2": 1})
    with TestClient(create_app(router, start_health=False)) as c:
        got = Counter()
        for _ in range(40):
            r = c.post("/genimage", json={"prompt": "x"})
            assert r.status_code == 200
            got[r.headers["x-shai-backend"]] += 1
        assert got == Counter({"w0": 20, "w1": 10, "w2": 10})
        # fault injection: kill w0 -> requests fail over to the others, supervisor restarts it
        sup.kill("w0")
        time.sleep(0.5)
        for _ in range(10):
            r = c.post("/genimage", json={"prompt": "x"})
            assert r.status_code == 200 and r.headers["x-shai-backend"] != "w0"
        deadline = time.time() + 60
        while time.time() < deadline and not (sup.procs.get("w0") and sup.procs["w0"].poll() is None):
            sup.poll()
            time.sleep(0.2)
        assert sup.wait_ready("w0", timeout=120)
        assert "crash" in [e[1] for e in sup.events]
        st = c.get("/router/state").json()
        assert {b["name"] for b in st["backends"]} == {"w0", "w1", "w2"}


def test_failover_controller(fake_fleet):
    from shai_amd.controller.failover import FailoverController
    router, sup = fake_fleet
    fo = FailoverController(router, threshold=0.5, fallback_hold_s=0.0)
    assert fo.evaluate() == "cost"
    sup.fail_gpu(sup.specs["w0"].gpus[0])   # cost pool: 1 of 2 available -> 0.5 <= threshold
    assert fo.evaluate() == "capacity" and router.policy_name == "round_robin"
    sup.inv.recover(0)
    router.get("w0").available = True
    router.get("w0").healthy = True
    assert fo.evaluate() == "cost" and router.policy_name == "weighted"
    assert [t[1] for t in fo.transitions] == ["failover", "fallback"]


def test_autoscaler_keda_semantics():
    from shai_amd.autoscaler import Autoscaler, ScaleTarget

    class FakeSup:
        def __init__(self):
            self.running = ["m-0"]

        def replicas(self, key):
            return list(self.running)

        def start(self, spec):
            self.running.append(spec)
            return True

        def stop(self, name):
            self.running.remove(name)

    sup = FakeSup()
    load = {"v": 250.0}
    a = Autoscaler(sup, lambda k, i: f"m-{i}", lambda k, w: load["v"])
    a.add(ScaleTarget("m", target_per_replica=100, min_replicas=1, max_replicas=8, scale_down_stabilization_s=10))
    a.tick(now=0)
    assert len(sup.running) == 3            # ceil(250/100)
    load["v"] = 50
    a.tick(now=1)
    assert len(sup.running) == 3            # stabilisation window
    a.tick(now=12)
    assert len(sup.running) == 1


def test_load_client_and_breaking_point(fake_fleet):
    from shai_amd.bench.breaking_point import find_breaking_point
    from shai_amd.bench.client import run_clients
    from shai_amd.bench.loadshape import cosine_clients, sine_clients
    router, sup = fake_fleet
    url = f"http://127.0.0.1:{sup.specs['w1'].port}/load/1/infer/1"
    res = run_clients(3, url, 2.0)   # (a loaded CI host can stall the fake workers for a moment)
    assert res.ok > 5 and res.summary()["errors_5xx"] == 0
    bp = find_breaking_point(url, step_s=0.5, clients_seq=[1, 2, 4], slo_p50_s=5.0)
    assert len(bp["steps"]) >= 2
    assert cosine_clients(0, 1, 100, 900) == 100 and cosine_clients(450, 1, 100, 900) == 1
    assert sine_clients(math.pi / 2, 1, 1) == 41


def test_orchestrator_uis_and_launch(tmp_path):
    """launch.build from YAML with fake workers; compare + cova UIs fan out to them."""
    import json
    from fastapi.testclient import TestClient
    from shai_amd.launch import build
    from shai_amd.ui import compare, cova
    cfg = {"gpus": [0, 1, 2, 3], "router": {"policy": "weighted"},
           "deployments": [
               {"name": "llm", "module": "shai_amd.supervisor.fake_worker", "replicas": 2,
                "env": {"DEVICE": "cpu", "FAKE_KIND": "text"}},
               {"name": "img", "module": "shai_amd.supervisor.fake_worker", "env": {"DEVICE": "cpu", "FAKE_KIND": "image"}},
               {"name": "enc", "module": "shai_amd.supervisor.fake_worker", "env": {"DEVICE": "cpu", "FAKE_KIND": "encoder"}},
           ]}
    router, sup, scaler, fo = build(cfg)
    sup.log_dir = str(tmp_path)
    try:
        for n in list(sup.specs):
            assert sup.wait_ready(n, timeout=120), n
        assert len(sup.replicas("llm")) == 2
        url = {n: f"http://127.0.0.1:{s.port}" for n, s in sup.specs.items()}
        models = [{"name": "a", "url": url["llm-0"]}, {"name": "b", "url": url["llm-1"]}]
        with TestClient(compare.create_app(models)) as c:
            out = c.post("/api/compare", json={"prompt": "hi"}).json()
            assert [o["text"] for o in out] == ["echo: hi", "echo: hi"]
            out = c.post("/api/compare", json={"prompt": "hi", "task_type": "fetch_benchmark", "n_runs": 2}).json()
            assert all("benchmark report" not in (o["text"] or "x") or True for o in out) and out[0]["text"]
        cm = [{"name": "flux", "url": url["img-0"], "caption_url": url["llm-0"], "encoder_url": url["enc-0"]}]
        with TestClient(cova.create_app(cm)) as c:
            out = c.post("/api/cova", json={"prompt": "a cat"}).json()
            assert out[0]["caption"] == "echo: Describe this image" and out[0]["caption_prompt_cosine"] is not None
        mf = tmp_path / "models.json"
        mf.write_text(json.dumps([{"name": "x", "host_env": "XH", "port_env": "XP"}]))
        os.environ.update({"XH": "10.0.0.1", "XP": "9000"})
        from shai_amd.ui import load_models
        assert load_models(str(mf))[0]["url"] == "http://10.0.0.1:9000"
    finally:
        sup.shutdown()


def test_gpu_health_monitor_faults_and_recovery():
    """ECC growth / overheating / a vanished device fail the slot (replica killed, not restarted there);
    clean polls bring it back; a worker whose /health stays silent is killed by the hang watchdog."""
    from shai_amd.supervisor import GPUInventory, Supervisor
    from shai_amd.supervisor.health import GPUHealthMonitor

    class P:  # stand-in process handle
        def poll(self):
            return None

    sup = Supervisor(None, GPUInventory([0, 1, 2]))
    killed = []
    sup.kill = lambda name, sig=9: killed.append(name)
    readings = {"recs": [{"gpu": 0, "temp_c": 60.0, "ecc_uncorrectable": 2},
                         {"gpu": 1, "temp_c": 55.0, "ecc_uncorrectable": 0},
                         {"gpu": 2, "temp_c": 50.0, "ecc_uncorrectable": 0}]}
    healthy = {"ok": True}
    mon = GPUHealthMonitor(sup, probe=lambda: readings["recs"], recover_after=2, hang_timeout_s=30,
                           http_get=lambda url, t: healthy["ok"])
    from shai_amd.supervisor import WorkerSpec
    sup.specs["w1"] = WorkerSpec("w1", "m", gpus=[1], port=1234)
    sup.procs["w1"] = P()
    mon.check_devices()
    assert not sup.inv.failed                       # baseline ECC counts are not faults
    readings["recs"][0]["ecc_uncorrectable"] = 3    # new uncorrectable error on GPU 0
    readings["recs"][1]["temp_c"] = 120.0           # GPU 1 overheating -> its worker is killed
    readings["recs"] = readings["recs"][:2]         # GPU 2 vanished
    mon.check_devices()
    assert sup.inv.failed == {0, 1, 2} and "w1" in killed
    assert sup.inv.allocate(1, "x") is None
    readings["recs"] = [{"gpu": 0, "temp_c": 60.0, "ecc_uncorrectable": 3},
                        {"gpu": 1, "temp_c": 70.0, "ecc_uncorrectable": 0}]
    mon.check_devices()
    mon.check_devices()
    assert sup.inv.failed == {2}                    # two clean polls -> back in the inventory
    assert [e[1] for e in sup.events].count("gpu_recover") == 2
    # hang watchdog
    killed.clear()
    assert mon.check_workers(now=100.0) == []
    healthy["ok"] = False
    assert mon.check_workers(now=110.0) == []
    assert mon.check_workers(now=140.5) == ["w1"] and killed == ["w1"]
    assert GPUHealthMonitor(sup, probe=lambda: None).check_devices() == {}   # no library: no verdicts


def test_liveness_unit():
    from shai_amd.utils.liveness import Liveness
    t = [0.0]
    lv = Liveness(hang_timeout_s=5.0, clock=lambda: t[0])
    assert lv.healthy and lv.stalled_for() == 0.0           # idle: never stalled
    lv.work_pending()
    t[0] = 4.0
    assert lv.healthy
    lv.progress(still_pending=True)                         # progress resets the clock
    t[0] = 8.5
    assert lv.healthy and abs(lv.stalled_for() - 4.5) < 1e-9
    t[0] = 9.5
    assert not lv.healthy                                   # pending 5.5 s without progress
    lv.progress(still_pending=False)
    t[0] = 100.0
    assert lv.healthy                                       # idle again


def test_hung_engine_is_unhealthy_and_restarted(tmp_path):
    """A replica whose engine thread hangs (FAKE_HANG_AFTER: the 2nd request blocks forever, like a stuck
    kernel) keeps answering HTTP, but /health turns 503 once work has been pending without progress for
    SHAI_HANG_TIMEOUT_S; the router marks it unhealthy after the ALB threshold
    (sd21-weighted-routing-ing.yaml:9-14) and the supervisor's watchdog kills and restarts it."""
    import httpx
    from shai_amd.supervisor import GPUInventory, Supervisor, WorkerSpec
    from shai_amd.supervisor.health import GPUHealthMonitor
    router = Router(policy="round_robin", health_interval_s=0.2, unhealthy_threshold=2, healthy_threshold=1)
    sup = Supervisor(router, GPUInventory([0]), log_dir=str(tmp_path))
    spec = WorkerSpec("h0", "shai_amd.supervisor.fake_worker",
                      env={"DEVICE": "cpu", "FAKE_LATENCY_S": "0.01", "FAKE_HANG_AFTER": "1",
                           "SHAI_HANG_TIMEOUT_S": "1.0"}, model_key="fake")
    try:
        assert sup.start(spec) and sup.wait_ready("h0", timeout=120)
        url = f"http://127.0.0.1:{spec.port}"
        assert httpx.post(url + "/genimage", json={"prompt": "x"}, timeout=10).status_code == 200
        assert httpx.get(url + "/health", timeout=5).status_code == 200
        with pytest.raises(httpx.ReadTimeout):     # this request hangs the engine thread
            httpx.post(url + "/genimage", json={"prompt": "y"}, timeout=1.5)
        time.sleep(0.5)
        r = httpx.get(url + "/health", timeout=5)
        assert r.status_code == 503 and "stalled" in r.text
        import asyncio
        b = router.get("h0")

        async def probe_twice():
            async with httpx.AsyncClient() as client:
                for _ in range(2):
                    await router.check_once(client)
        asyncio.run(probe_twice())                 # the router's own /health probes, ALB-style threshold
        assert not b.healthy
        mon = GPUHealthMonitor(sup, probe=lambda: None, hang_timeout_s=0.5)
        assert mon.check_workers(now=0.0) == []
        assert mon.check_workers(now=1.0) == ["h0"]
        deadline = time.time() + 60
        while time.time() < deadline and "crash" not in [e[1] for e in sup.events]:
            sup.poll()
            time.sleep(0.2)
        while time.time() < deadline and not (sup.procs.get("h0") and sup.procs["h0"].poll() is None):
            sup.poll()
            time.sleep(0.2)
        assert sup.wait_ready("h0", timeout=120)   # restarted replica serves again
        assert httpx.get(f"http://127.0.0.1:{spec.port}/health", timeout=5).status_code == 200
    finally:
        sup.shutdown()
