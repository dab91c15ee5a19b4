"""Model-free worker speaking the SD/LLM API (for router / supervisor /
autoscaler tests and load-generator dry runs): configurable latency
(FAKE_LATENCY_S), failure injection (FAKE_FAIL_RATE) and a hung engine
(FAKE_HANG_AFTER=n: the engine thread blocks forever on request n + 1, the way a
hung kernel blocks a real engine; ``/health`` then turns 503 after
SHAI_HANG_TIMEOUT_S)."""
import os
import random
import time

import threading

from ..serving.common import METRICS, EngineWorker, ServerEnv, base_app, benchmark, run


def create_app():
    env = ServerEnv.from_env(app=os.environ.get("APP", "fake"))
    lat = float(os.environ.get("FAKE_LATENCY_S", "0.01"))
    fail = float(os.environ.get("FAKE_FAIL_RATE", "0"))
    hang_after = int(os.environ.get("FAKE_HANG_AFTER", "-1"))
    app = base_app(env, "fake worker", spaced=False)
    engine = EngineWorker("fake-engine")
    served = [0]

    def _engine_work():
        served[0] += 1
        if 0 <= hang_after < served[0]:
            threading.Event().wait()   # never returns: a stuck kernel
        time.sleep(lat)
        if random.random() < fail:
            raise RuntimeError("injected failure")

    def work():
        return engine.call(_engine_work)

    @app.post("/genimage")
    def genimage(request: dict):
        t0 = time.time()
        work()
        METRICS.request_done(env, time.time() - t0)
        return {"prompt": request.get("prompt"), "response": "", "latency": str(time.time() - t0),
                "pod": env.pod_name}

    @app.post("/generate")
    def generate(request: dict):
        """LLM / encoder / image-gen shaped response (FAKE_KIND = text | encoder | image)."""
        import base64
        t0 = time.time()
        work()
        kind = os.environ.get("FAKE_KIND", "text")
        prompt = request.get("prompt", "")
        if kind == "encoder":
            txt = "[" + " ".join(f"{(hash(prompt) >> (4 * i)) % 7 / 7:.3f}" for i in range(8)) + "]"
            out = {"text": base64.b64encode(txt.encode()).decode()}
        elif kind == "image":
            from ..serving.common import png_b64
            import numpy as np
            out = {"image": png_b64(np.zeros((8, 8, 3), np.uint8))}
        else:
            out = {"text": base64.b64encode(f"echo: {prompt}".encode()).decode()}
        out["prompt"], out["execution_time"] = prompt, time.time() - t0
        METRICS.request_done(env, time.time() - t0)
        return out

    @app.post("/benchmark")
    def bench(request: dict):
        import base64
        rep = benchmark(int(request.get("n_runs", 1)), "fake", work, env.pod_name)
        return {"report": base64.b64encode(rep.encode()).decode(), "execution_time": 0.0}

    @app.get("/load/{n_runs}/infer/{n_inf}")
    def load(n_runs: int, n_inf: int):
        return {"message": "benchmark report:" + benchmark(n_runs, "stable_diffusion_512", work, env.pod_name)}

    return app


if __name__ == "__main__":
    run(create_app())
