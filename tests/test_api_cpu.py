"""API contract tests: every reference endpoint on tiny CPU models
via FastAPI's TestClient -- paths, JSON keys, types, base64 payloads, report format."""
import base64
import io
import re

import numpy as np
import pytest
from fastapi.testclient import TestClient

from shai_amd.serving.common import LatencyCollector, ServerEnv, latency_report

REPORT_RE = re.compile(r"RESULT FOR .+: Latency P0=\d+\.\d Latency P50=\d+\.\d Latency P90=\d+\.\d "
                       r"Latency P95=\d+\.\d Latency P99=\d+\.\d Latency P100=\d+\.\d$")


def env(**kw):
    base = dict(app="t", pod_name="pod0", nodepool="mi355x", model_id="m", device="cpu", config="tiny",
                num_inference_steps=2, max_new_tokens=4, max_seq_len=16, height=64, width=64)
    base.update(kw)
    return ServerEnv(**base)


def test_percentile_rule_matches_reference():
    lc = LatencyCollector()
    lc.latency_list = [0.5, 0.1, 0.3, 0.2, 0.4]
    assert lc.percentile(0) == 0.1 and lc.percentile(100) == 0.5
    assert lc.percentile(50) == 0.3   # pos 2.5 -> floor (frac not > .5)
    assert lc.percentile(90) == 0.5   # pos 4.5 -> floor 4
    lc.latency_list = [1, 2, 3, 4, 5, 6, 7]
    assert lc.percentile(90) == 7     # pos 6.3 -> floor 6
    assert lc.percentile(95) == 7     # 6.65 -> ceil clipped
    r = latency_report(lc, "stable_diffusion_512", "pod0")
    assert r.startswith("RESULT FOR stable_diffusion_512 on pod0: Latency P0=1000.0") and REPORT_RE.match(r)


def test_sd_server():
    from shai_amd.serving import sd
    c = TestClient(sd.create_app(env=env(app="sd21")))
    assert c.get("/health").json() == {"message": "pod0is healthy"}
    assert c.get("/readiness").json() == {"message": "pod0is ready"}
    assert c.get("/").json()["message"].startswith("This ism pod pod0")
    r = c.post("/genimage", json={"prompt": "a cat"}).json()
    assert set(r) == {"prompt", "response", "latency"} and isinstance(r["latency"], str)
    from PIL import Image
    im = Image.open(io.BytesIO(base64.b64decode(r["response"])))
    assert im.size == (64, 64)
    m = c.get("/load/2/infer/2").json()["message"]
    assert m.startswith("benchmark report:RESULT FOR stable_diffusion_512 on pod0:")
    assert REPORT_RE.match(m[len("benchmark report:"):])
    prom = c.get("/metrics").text
    assert "sd21_counter_total" in prom and "mi355x_total" in prom
    assert c.get("/serve").status_code == 200


def test_sd_server_rejects_bad_requests_alone():
    """A malformed request is a 422 for its own caller and never reaches the step-batching engine thread
    (steps < 1 would divide by zero in the schedule, a non-string prompt would fail the text encoder for every
    request regrouped with it); the server keeps serving."""
    from shai_amd.serving import sd
    c = TestClient(sd.create_app(env=env(app="sd21")))
    assert c.get("/load/1/infer/0").status_code == 422
    assert c.get("/load/1/infer/-3").status_code == 422
    assert c.post("/genimage", json={}).status_code == 422
    assert c.post("/genimage", json={"prompt": 5}).status_code == 422
    worker = c.app.state.worker
    import pytest as _pt
    with _pt.raises(ValueError):
        worker.submit("x", 0)
    assert worker.t.is_alive()
    assert c.post("/genimage", json={"prompt": "a cat"}).status_code == 200
    assert c.get("/health").status_code == 200


def test_broken_replica_health_is_503():
    """A fault the process cannot recover from in place (an xGMI peer collective that timed out, a dead TP
    rank) marks it broken for good: /health answers 503 so the router drains it and the supervisor restarts
    it, even though the engine loop itself keeps making 'progress' by failing requests."""
    from shai_amd.serving import bert
    from shai_amd.utils import liveness
    from shai_amd.parallel import comm
    c = TestClient(bert.create_app(env=env(app="bert", device="cpu")))
    assert c.get("/health").status_code == 200

    class _Err:
        def error(self):
            return True
    old = comm.p2p()
    comm.enable_p2p(_Err())
    try:
        import pytest as _pt
        with _pt.raises(RuntimeError, match="TP group broken"):
            comm.raise_if_p2p_error()
        r = c.get("/health")
        assert r.status_code == 503 and "broken" in r.text
        assert c.get("/health").status_code == 503     # permanent, not a one-off
    finally:
        comm.enable_p2p(old)
        liveness._reset_broken_for_tests()
    assert c.get("/health").status_code == 200


def test_llm_api_server():
    from shai_amd.serving import llm_api
    c = TestClient(llm_api.create_app(env=env(app="mistral")))
    assert c.get("/health").json() == {"message": "pod0 is healthy"}
    r = c.post("/generate", json={"prompt": "What model are you?", "max_new_tokens": 5}).json()
    assert set(r) == {"text", "execution_time"} and isinstance(r["execution_time"], float)
    base64.b64decode(r["text"]).decode()
    # multimodal variant: optional base64 image
    from PIL import Image
    buf = io.BytesIO()
    Image.new("RGB", (8, 8)).save(buf, format="PNG")
    r2 = c.post("/generate", json={"prompt": "describe", "max_new_tokens": 3,
                                   "image": base64.b64encode(buf.getvalue()).decode()})
    assert r2.status_code == 200
    rep = base64.b64decode(c.post("/benchmark", json={"n_runs": 3, "max_new_tokens": 4, "prompt": "hi"}).json()
                           ["report"]).decode()
    assert rep.startswith("RESULT FOR benchmark:mistral on mi355x with 4 output tokens: Latency P0=")


def test_llm_api_multimodal_server():
    """Llama-3.2-Vision (tiny) behind the vllm_model_api_m.py schema: the image is attended to."""
    from shai_amd.serving import llm_api
    c = TestClient(llm_api.create_app(env=env(app="mllama", model_id="meta-llama/Llama-3.2-11B-Vision-Instruct")))
    svc = c.app.state.service
    assert svc.multimodal
    r = c.post("/generate", json={"prompt": "Describe this image", "max_new_tokens": 3, "image": _img_b64()})
    assert r.status_code == 200 and set(r.json()) == {"text", "execution_time"}
    ids = svc.encode(llm_api.add_instruct("Describe this image", True))
    assert ids.count(svc.engine.mcfg.image_token_index) == 1 and ids[0] == svc.engine.cfg.bos_token_id
    assert svc.engine.bm.num_free == svc.engine.num_kv_blocks


def test_llm_gradio_server():
    from shai_amd.serving import llm_gradio
    c = TestClient(llm_gradio.create_app(env=env(app="llama")))
    r = c.post("/gentext", json={"prompt": "write a poem"}).json()
    assert set(r) == {"prompt", "response", "latency"} and isinstance(r["latency"], str)
    r = c.post("/sentiment", json={"prompt": "great movie"}).json()
    assert set(r) == {"prompt", "response", "latency"}
    assert c.get("/health").json() == {"message": "pod0is healthy"}


def test_bert_server():
    from shai_amd.serving import bert
    c = TestClient(bert.create_app(env=env(app="bert")))
    r = c.post("/sentiment", json={"prompt": "Hamilton is great"}).json()
    assert r["response"] in ("POSITIVE", "NEGATIVE") and isinstance(r["latency"], float)
    assert c.options("/sentiment", headers={"Origin": "http://x", "Access-Control-Request-Method": "POST"}
                     ).headers.get("access-control-allow-origin") in ("*", "http://x")


def _img_b64(w=96, h=80):
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray((np.random.default_rng(0).random((h, w, 3)) * 255).astype(np.uint8)).save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


def test_vit_server():
    from shai_amd.serving import vit
    c = TestClient(vit.create_app(env=env(app="vit")))
    src = _img_b64()
    r = c.post("/imgcls", json={"prompt": src}).json()
    assert r["image"] == src and r["response"].startswith("LABEL_") and isinstance(r["latency"], float)


def test_yolos_server():
    from shai_amd.serving import yolos
    c = TestClient(yolos.create_app(env=env(app="yolos")))
    r = c.post("/detectobj", json={"prompt": _img_b64()}).json()
    assert set(r) == {"image", "response", "latency"} and isinstance(r["response"], list)
    for d in r["response"]:
        assert set(d) == {"score", "label", "box"} and set(d["box"]) == {"xmin", "ymin", "xmax", "ymax"}


def test_t5_server():
    from shai_amd.serving import t5_api
    c = TestClient(t5_api.create_app(env=env(app="t5")))
    r = c.post("/generate", json={"prompt": "a caption", "max_new_tokens": 16}).json()
    txt = base64.b64decode(r["text"]).decode()
    assert txt.startswith("[") and isinstance(r["execution_time"], float)
    rep = base64.b64decode(c.post("/benchmark", json={"n_runs": 2, "max_new_tokens": 16, "prompt": "x"}).json()
                           ["report"]).decode()
    assert rep.startswith("RESULT FOR benchmark:t5 on mi355x with 16 output tokens:")


def test_flux_servers():
    from PIL import Image
    from shai_amd.serving import flux_api
    e = env(app="flux", model_id="black-forest-labs/FLUX.1-dev")
    eng = flux_api.build_engine(e)
    c = TestClient(flux_api.create_app(engine=eng, env=e))
    assert c.get("/health").json() == {"message": "pod0 is healthy"}
    assert c.get("/readiness").json() == {"message": "pod0 is ready"}
    r = c.post("/generate", json={"prompt": "a cat", "num_inference_steps": 2})
    assert r.status_code == 200
    j = r.json()
    assert set(j) == {"image", "execution_time"} and isinstance(j["execution_time"], float)
    im = Image.open(io.BytesIO(base64.b64decode(j["image"])))
    assert max(im.size) <= 128
    bad = c.post("/generate", json={"prompt": "a cat", "num_inference_steps": -1})
    assert bad.status_code == 500 and bad.json()["detail"].startswith("Image serialization failed: ")
    g = TestClient(flux_api.create_gradio_app(engine=eng, env=e))
    assert g.get("/health").json() == {"message": "pod0is healthy"}
    j = g.post("/text2img", json={"prompt": "a dog", "num_inference_steps": 2}).json()
    assert isinstance(j["execution_time"], str)
    assert Image.open(io.BytesIO(base64.b64decode(j["image"]))).size == (64, 64)
    assert g.get("/serve").status_code == 200


def test_flux_engine_tiny_deterministic():
    import torch
    from shai_amd.engines.flux import FluxEngine, FluxPipelineConfig
    eng = FluxEngine(FluxPipelineConfig.tiny(), device="cpu")
    a = eng.generate(["a red fox"], 3, seed=7)
    b = eng.generate(["a red fox"], 3, seed=7)
    assert a.shape == (1, 64, 64, 3) and a.dtype == torch.uint8 and torch.equal(a, b)
