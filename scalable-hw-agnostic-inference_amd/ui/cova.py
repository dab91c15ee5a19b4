"""Content-validation chain (app/cova_gradio_m.py + cova/*.yaml): for every
configured resolution, Flux /generate -> multimodal LLM caption (/generate with
the image) -> T5 embeddings of the caption and of the prompt, with per-stage
latencies; all models in parallel (asyncio.gather), each chain sequential.
  POST /api/cova {"prompt": str, "num_inference_steps": int}
"""
import asyncio
import base64
import io

import numpy as np

from . import load_models


async def post_json(client, url, payload, timeout=600.0):
    loop = asyncio.get_event_loop()
    t0 = loop.time()
    r = await client.post(url, json=payload, timeout=timeout)
    r.raise_for_status()
    return r.json(), loop.time() - t0


def parse_embedding(s: str) -> np.ndarray:
    return np.array([float(x) for x in s.replace("[", " ").replace("]", " ").split()], dtype=np.float32)


async def fetch_end_to_end(client, m, prompt, steps):
    img_json, img_lat = await post_json(client, m["url"] + "/generate", {"prompt": prompt,
                                                                          "num_inference_steps": int(steps)})
    cap_json, cap_lat = await post_json(client, m["caption_url"] + "/generate", {
        "prompt": "Describe this image", "image": img_json["image"],
        "max_new_tokens": m.get("caption_max_new_tokens", 128)})
    caption = base64.b64decode(cap_json["text"]).decode()
    mnt = m.get("encoder_max_new_tokens", 256)
    enc_cap, enc_cap_lat = await post_json(client, m["encoder_url"] + "/generate",
                                           {"prompt": caption, "max_new_tokens": mnt})
    enc_p, enc_p_lat = await post_json(client, m["encoder_url"] + "/generate", {"prompt": prompt, "max_new_tokens": mnt})
    e1 = parse_embedding(base64.b64decode(enc_cap["text"]).decode())
    e2 = parse_embedding(base64.b64decode(enc_p["text"]).decode())
    cos = float(e1 @ e2 / (np.linalg.norm(e1) * np.linalg.norm(e2) + 1e-9)) if e1.size == e2.size else None
    return {"name": m.get("name"), "image": img_json["image"], "image_latency": f"{img_lat:.2f}s",
            "caption": caption, "caption_latency": f"{cap_lat:.2f}s",
            "caption_embedding_latency": f"{enc_cap_lat:.2f}s", "prompt_embedding_latency": f"{enc_p_lat:.2f}s",
            "caption_prompt_cosine": cos}


def create_app(models=None):
    import httpx
    from fastapi import FastAPI
    from fastapi.responses import HTMLResponse
    models = models if models is not None else load_models()
    app = FastAPI(title="cova")

    @app.post("/api/cova")
    async def cova(body: dict):
        async with httpx.AsyncClient() as client:
            return await asyncio.gather(*(fetch_end_to_end(client, m, body.get("prompt", ""),
                                                           body.get("num_inference_steps", 10)) for m in models))

    @app.get("/serve", response_class=HTMLResponse)
    def serve():
        return ("<html><body><h3>Flux image-gen + caption + T5 embeddings</h3><input id=p size=80>"
                "<button onclick=\"fetch('/api/cova',{method:'POST',headers:{'Content-Type':'application/json'},"
                "body:JSON.stringify({prompt:document.getElementById('p').value,num_inference_steps:10})}).then(r=>"
                "r.json()).then(j=>{document.getElementById('i').src='data:image/png;base64,'+j[0].image;"
                "j.forEach(x=>delete x.image);document.getElementById('o').textContent=JSON.stringify(j,null,2)})\">"
                "Generate</button><br><img id=i><pre id=o></pre></body></html>")

    @app.get("/health")
    def health():
        return {"message": "cova is healthy"}

    return app
