"""Offline harnesses on tiny CPU models: the mllama-offline.py counterpart (4 prompt/image/sampling combos,
percentile report) and the app/src/inference.py counterpart (standalone Flux run writing a PNG)."""
import os
import re


def test_llm_offline_multimodal_tiny(capsys):
    from shai_amd.bench import llm_offline
    llm_offline.main(["--config", "tiny", "--rounds", "2", "--max-tokens-cap", "3", "--device", "cpu"])
    out = capsys.readouterr().out
    assert re.search(r"RESULT FOR MLLAMA: Latency P0=\d+\.\d .* Latency P100=\d+\.\d", out)


def test_llm_offline_concurrent_text_model(capsys):
    from shai_amd.bench import llm_offline
    llm_offline.main(["--model", "mistralai/Mistral-7B-Instruct-v0.3", "--config", "tiny", "--rounds", "1",
                      "--max-tokens-cap", "2", "--concurrent", "--device", "cpu"])
    assert "RESULT FOR LLM:" in capsys.readouterr().out


def test_flux_offline_tiny(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import flux_offline
    out = tmp_path / "flux.png"
    img = flux_offline.main(["--config", "tiny", "-n", "2", "--out", str(out), "--device", "cpu"])
    assert out.exists() and img.shape == (1, 64, 64, 3)
