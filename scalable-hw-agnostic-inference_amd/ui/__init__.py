"""Orchestrator UIs (Gradio is not installed in this image: each UI is a FastAPI
app with a JSON API plus a minimal HTML page at /serve)."""
import json
import os


def load_models(path=None):
    """models.json (MODELS_FILE_PATH); host/port come from the named env vars
    (K8s service env in the reference), or direct "url" entries."""
    path = path or os.environ.get("MODELS_FILE_PATH", "")
    if not path or not os.path.exists(path):
        return []
    with open(path) as f:
        models = json.load(f)

    def url(m, host_key, port_key):
        if host_key in m and port_key in m:
            return f"http://{os.environ.get(m[host_key], '127.0.0.1')}:{os.environ.get(m[port_key], '8000')}"
        return None

    for m in models:
        m.setdefault("url", url(m, "host_env", "port_env"))
        if "caption_host_env" in m:
            m.setdefault("caption_url", url(m, "caption_host_env", "caption_port_env"))
        if "encoder_host_env" in m:
            m.setdefault("encoder_url", url(m, "encoder_host_env", "encoder_port_env"))
    return models
