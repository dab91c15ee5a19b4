"""Tensor-parallel serving end to end on CPU: the supervisor launches a server as a TP=2 group
(``torch.distributed.run``, gloo), rank 0 answers HTTP and mirrors every engine call / LLM step to rank 1
(serving/tp.py).  Each TP2 answer is compared with the same server at TP1.

Reference: app/vllm_model_api.py:127-129 (LLM(**vllm_config), tensor_parallel_size),
app/flux_model_api.py:128-140,312-314 (Flux transformer / T5 TP8), app/t5_model_api.py:27,33."""
import base64
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.slow


def _fleet(tmp_path, module, extra_env, tps=(1, 2), restart=False):
    from shai_amd.supervisor import GPUInventory, Supervisor, WorkerSpec
    sup = Supervisor(None, GPUInventory(list(range(2 * len(tps)))), log_dir=str(tmp_path))  # slots, not GPUs
    env = {"DEVICE": "cpu", "SHAI_MODEL_CONFIG": "tiny", "OMP_NUM_THREADS": "2", "SHAI_TP_HEARTBEAT_S": "1"}
    env.update(extra_env)
    names = []
    for tp in tps:
        spec = WorkerSpec(f"{module.rsplit('.', 1)[-1]}-tp{tp}", module, tp=tp, env=dict(env), restart=restart)
        assert sup.start(spec)
        names.append(spec.name)
    for n in names:
        ok = sup.wait_ready(n, timeout=600)
        assert ok, open(os.path.join(tmp_path, f"{n}.log")).read()[-4000:]
    return sup, names


def _post(sup, name, path, body, timeout=300):
    import httpx
    r = httpx.post(f"http://127.0.0.1:{sup.specs[name].port}{path}", json=body, timeout=timeout)
    assert r.status_code == 200, r.text
    return r.json()


def _get(sup, name, path):
    import httpx
    return httpx.get(f"http://127.0.0.1:{sup.specs[name].port}{path}", timeout=30)


def test_llm_api_tp2_matches_tp1(tmp_path):
    sup, (n1, n2) = _fleet(tmp_path, "shai_amd.serving.llm_api", {"SHAI_TEMPERATURE": "0"})
    try:
        texts = {}
        for n in (n1, n2):
            out = _post(sup, n, "/generate", {"prompt": "the quick brown fox", "max_new_tokens": 12})
            texts[n] = base64.b64decode(out["text"]).decode()
            assert out["execution_time"] > 0
            # concurrent requests share engine steps: the follower must mirror every admission
            import concurrent.futures as cf
            with cf.ThreadPoolExecutor(4) as ex:
                outs = list(ex.map(lambda p: _post(sup, n, "/generate", {"prompt": p, "max_new_tokens": 6}),
                                   ["a", "bb cc", "dd ee ff", "the quick brown fox"]))
            assert base64.b64decode(outs[3]["text"]).decode() == texts[n][:len(base64.b64decode(outs[3]["text"]).decode())]
            h = _get(sup, n, "/health")
            assert h.status_code == 200 and "is healthy" in h.json()["message"]
            rep = _post(sup, n, "/benchmark", {"n_runs": 2, "max_new_tokens": 4, "prompt": "hi"})
            assert base64.b64decode(rep["report"]).decode().startswith("RESULT FOR benchmark:")
        assert texts[n1] == texts[n2], (texts[n1], texts[n2])
        log = open(os.path.join(tmp_path, f"{n2}.log")).read()
        assert "tp_up" in log
    finally:
        sup.shutdown()


def _png(b64):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(base64.b64decode(b64))).convert("RGB")).astype(np.float32)


def test_flux_api_tp2_matches_tp1(tmp_path):
    sup, (n1, n2) = _fleet(tmp_path, "shai_amd.serving.flux_api", {"FLUX_WARMUP_RUNS": "1", "SHAI_SEED": "7"})
    try:
        imgs = {}
        for n in (n1, n2):
            out = _post(sup, n, "/generate", {"prompt": "a cat", "num_inference_steps": 2})
            imgs[n] = _png(out["image"])
            assert imgs[n].shape[-1] == 3
        # same weights (seeded random init), same seed: the TP2 image is the TP1 image up to bf16 rounding
        assert imgs[n1].shape == imgs[n2].shape
        assert np.abs(imgs[n1] - imgs[n2]).mean() < 4.0, np.abs(imgs[n1] - imgs[n2]).mean()
        assert _get(sup, n2, "/health").status_code == 200
    finally:
        sup.shutdown()


def test_t5_api_tp2_matches_tp1(tmp_path):
    sup, (n1, n2) = _fleet(tmp_path, "shai_amd.serving.t5_api", {})
    try:
        embs = {}
        for n in (n1, n2):
            out = _post(sup, n, "/generate", {"prompt": "a caption of a cat", "max_new_tokens": 16})
            txt = base64.b64decode(out["text"]).decode()
            embs[n] = np.array([float(v) for v in txt.strip("[] \n").split()])
        a, b = embs[n1], embs[n2]
        assert a.shape == b.shape and a.size > 0
        assert np.linalg.norm(a - b) / (np.linalg.norm(a) + 1e-6) < 3e-2
    finally:
        sup.shutdown()


def test_llm_api_tp2_rank_failure_restarts_group(tmp_path):
    """Kill rank 1 of a supervisor-launched TP2 LLM server: rank 0 turns unhealthy (503, or gone) within the ALB
    check budget (sd21-weighted-routing-ing.yaml:9-14: 10 s interval x 10 failures), the launcher tears the group
    down, and the supervisor relaunches it whole; the relaunched group serves again."""
    import time
    sup, (n2,) = _fleet(tmp_path, "shai_amd.serving.llm_api", {"SHAI_TEMPERATURE": "0"}, tps=(2,), restart=True)
    sup.monitor(0.5)
    try:
        first = base64.b64decode(_post(sup, n2, "/generate", {"prompt": "hello", "max_new_tokens": 4})["text"])
        pids = sup.rank_pids(n2)
        assert set(pids) == {0, 1}, pids
        t0 = time.time()
        assert sup.kill_rank(n2, 1)

        def health():
            try:
                return _get(sup, n2, "/health").status_code
            except Exception:  # noqa: BLE001 -- the leader is gone
                return None
        while health() == 200:
            assert time.time() - t0 < 100, "rank 0 still healthy after its follower died"
            time.sleep(0.2)
        t_unhealthy = time.time() - t0
        # relaunched as a group: new PIDs for both ranks, healthy again, same answer
        deadline = time.time() + 600
        while True:
            new = sup.rank_pids(n2)
            if set(new) == {0, 1} and all(new[r] != pids[r] for r in (0, 1)) and health() == 200:
                break
            assert time.time() < deadline, open(os.path.join(tmp_path, f"{n2}.log")).read()[-4000:]
            time.sleep(0.5)
        again = base64.b64decode(_post(sup, n2, "/generate", {"prompt": "hello", "max_new_tokens": 4})["text"])
        assert again == first
        assert sup.restarts.get(n2, 0) >= 1
        assert t_unhealthy < 100, t_unhealthy
    finally:
        sup.shutdown()
