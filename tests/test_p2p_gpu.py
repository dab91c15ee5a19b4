"""Custom xGMI/IPC one-shot all-reduce (csrc/comm/p2p_allreduce.hip), two ranks sharing cuda:0."""
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4, 8])
def test_p2p_allreduce_allgather_ranks_one_gpu(cuda, world):
    """One-shot / two-shot all-reduce, all-gather and graph replay with 2, 4 and 8 ranks (the TP degrees of
    app/src/transformer/compile.py:25) sharing one GPU through IPC."""
    import p2p_worker
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(p2p_worker.run, args=(world, port), nprocs=world, join=True)


def test_row_parallel_overlap_two_ranks_one_gpu(cuda):
    import tp_overlap_worker
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(tp_overlap_worker.run, args=(2, port), nprocs=2, join=True)


def test_tp2_llm_engine_on_p2p_one_gpu(cuda):
    """TP=2 LLM engine (two ranks on one GPU, P2P collectives on by default) vs TP=1: prefill + teacher-forced
    decode logits, HIP-graph decode, async look-ahead == sync tokens."""
    import tp_gpu_worker
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(tp_gpu_worker.run, args=(2, port), nprocs=2, join=True)


def test_tp2_flux_pipeline_on_p2p_one_gpu(cuda):
    import tp_gpu_worker
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(tp_gpu_worker.run_flux, args=(2, port), nprocs=2, join=True)


def test_llm_api_tp2_server_one_gpu(cuda, tmp_path):
    """The llm_api server launched as a TP=2 group (torch.distributed.run, both ranks on cuda:0, gloo control
    + P2P data): rank 0 answers /generate and /health; the answer equals the TP=1 server's greedy text."""
    import base64
    import os
    import subprocess
    import sys
    import time

    import httpx
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def start(tp):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        env = dict(os.environ, PORT=str(port), HOST="127.0.0.1", SHAI_MODEL_CONFIG="tiny", SHAI_TEMPERATURE="0",
                   TENSOR_PARALLEL_SIZE=str(tp), SHAI_TP_BACKEND="gloo", PYTHONPATH=root, POD_NAME=f"tp{tp}",
                   SHAI_P2P_MAX_BLOCKS="128", SHAI_P2P_TIMEOUT_S="10")
        env.pop("WORLD_SIZE", None)
        log = open(tmp_path / f"tp{tp}.log", "wb")
        p = subprocess.Popen([sys.executable, "-m", "shai_amd.serving.llm_api"], env=env, cwd=root, stdout=log,
                             stderr=subprocess.STDOUT, start_new_session=True)
        return p, port

    procs = []
    try:
        texts = {}
        for tp in (1, 2):
            p, port = start(tp)
            procs.append(p)
            deadline = time.time() + 240
            while time.time() < deadline:
                assert p.poll() is None, (tmp_path / f"tp{tp}.log").read_text()[-3000:]
                try:
                    if httpx.get(f"http://127.0.0.1:{port}/readiness", timeout=2).status_code == 200:
                        break
                except Exception:
                    pass
                time.sleep(0.5)
            else:
                raise AssertionError((tmp_path / f"tp{tp}.log").read_text()[-3000:])
            r = httpx.post(f"http://127.0.0.1:{port}/generate", json={"prompt": "the quick brown fox",
                                                                       "max_new_tokens": 8}, timeout=120)
            assert r.status_code == 200, r.text
            texts[tp] = base64.b64decode(r.json()["text"]).decode()
            assert httpx.get(f"http://127.0.0.1:{port}/health", timeout=5).status_code == 200
        assert texts[1] == texts[2], texts
    finally:
        import signal
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
                p.wait(timeout=30)
            except Exception:
                os.killpg(p.pid, signal.SIGKILL)
