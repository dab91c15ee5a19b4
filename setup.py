"""setuptools hook for pyproject.toml: lists the sub-packages of scalable-hw-agnostic-inference_amd/ under the
import name ``shai_amd`` and builds the gfx950 libraries (csrc/build.py, hipcc --offload-arch=gfx950) into
``_native/`` before they are copied into the wheel, when they are not built yet."""
import os
import subprocess
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = "scalable-hw-agnostic-inference_amd"
LIBS = ["libshai_kernels.so", "libshai_runtime.so", "libshai_comm.so"]


class BuildWithNative(build_py):
    def run(self):
        native = os.path.join(ROOT, PKG_DIR, "_native")
        if not all(os.path.exists(os.path.join(native, lib)) for lib in LIBS):
            subprocess.check_call([sys.executable, os.path.join(ROOT, "csrc", "build.py")])
        super().run()


SCRIPTS = {
    "shai-launch": "shai_amd.launch:main",
    "shai-serve-sd": "shai_amd.serving.sd:main",
    "shai-serve-flux": "shai_amd.serving.flux_api:main",
    "shai-serve-llm": "shai_amd.serving.llm_api:main",
    "shai-serve-llm-gradio": "shai_amd.serving.llm_gradio:main",
    "shai-serve-t5": "shai_amd.serving.t5_api:main",
    "shai-serve-bert": "shai_amd.serving.bert:main",
    "shai-serve-vit": "shai_amd.serving.vit:main",
    "shai-serve-yolos": "shai_amd.serving.yolos:main",
    "shai-breaking-point": "shai_amd.bench.breaking_point:main",
    "shai-load-client": "shai_amd.bench.client:main",
    "shai-loadshape": "shai_amd.bench.loadshape:main",
    "shai-llm-offline": "shai_amd.bench.llm_offline:main",
    "shai-long-context": "shai_amd.bench.long_context:main",
}

sub = find_packages(where=PKG_DIR)
setup(name="shai-amd", version="0.3.0",
      description="MI355X-native multi-model inference serving (SD2.1, Flux, Llama/Mistral, T5, BERT, ViT, YOLOS) "
                  "on hand-written gfx950 HIP kernels",
      python_requires=">=3.10",
      install_requires=["torch", "numpy", "fastapi", "uvicorn", "httpx", "pydantic", "pyyaml", "safetensors",
                        "pillow"],
      packages=["shai_amd"] + [f"shai_amd.{p}" for p in sub],
      package_dir={"shai_amd": PKG_DIR, **{f"shai_amd.{p}": os.path.join(PKG_DIR, *p.split(".")) for p in sub}},
      package_data={"shai_amd": ["_native/*.so"]},
      entry_points={"console_scripts": [f"{k} = {v}" for k, v in SCRIPTS.items()]},
      cmdclass={"build_py": BuildWithNative})
