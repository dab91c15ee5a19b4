"""Multi-model LLM comparison UI (app/llm_gradio.py): fans a prompt out to every
model's /generate (or /benchmark) concurrently and shows text + latency per model.
  POST /api/compare {"prompt", "task_type": "fetch_text"|"fetch_benchmark", "n_runs", "max_new_tokens"}
"""
import asyncio
import base64
import traceback

from . import load_models


async def fetch_text(client, url, prompt, max_new_tokens=32):
    try:
        r = await client.post(f"{url}/generate", json={"prompt": prompt, "max_new_tokens": max_new_tokens},
                              timeout=60.0)
        r.raise_for_status()
        d = r.json()
        return base64.b64decode(d["text"]).decode("utf-8"), f"{d.get('execution_time', 0):.2f} seconds"
    except Exception as e:
        traceback.print_exc()
        return None, f"Error: {e}"


async def fetch_benchmark(client, url, prompt, n_runs=1, max_new_tokens=32):
    try:
        r = await client.post(f"{url}/benchmark", json={"prompt": prompt, "n_runs": n_runs,
                                                        "max_new_tokens": max_new_tokens}, timeout=300.0)
        r.raise_for_status()
        d = r.json()
        return base64.b64decode(d["report"]).decode("utf-8"), f"{d.get('execution_time', 0):.2f} seconds"
    except Exception as e:
        traceback.print_exc()
        return None, f"Error: {e}"


def create_app(models=None):
    import httpx
    from fastapi import FastAPI
    from fastapi.responses import HTMLResponse
    models = models if models is not None else load_models()
    app = FastAPI(title="LLM compare")

    @app.post("/api/compare")
    async def compare(body: dict):
        prompt = body.get("prompt", "")
        n, mnt = int(body.get("n_runs", 1)), int(body.get("max_new_tokens", 32))
        async with httpx.AsyncClient() as client:
            if body.get("task_type", "fetch_text") == "fetch_benchmark":
                res = await asyncio.gather(*(fetch_benchmark(client, m["url"], prompt, n, mnt) for m in models))
            else:
                res = await asyncio.gather(*(fetch_text(client, m["url"], prompt, mnt) for m in models))
        return [{"name": m.get("name"), "text": t, "latency": lat} for m, (t, lat) in zip(models, res)]

    @app.get("/serve", response_class=HTMLResponse)
    def serve():
        return ("<html><body><h3>LLM compare</h3><input id=p size=80><button onclick=\"fetch('/api/compare',"
                "{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({prompt:"
                "document.getElementById('p').value})}).then(r=>r.json()).then(j=>document.getElementById('o')."
                "textContent=JSON.stringify(j,null,2))\">Go</button><pre id=o></pre></body></html>")

    @app.get("/health")
    def health():
        return {"message": "compare is healthy"}

    return app
