"""shai_amd -- MI355X-native multi-model inference serving stack.

Capabilities mirror ``vin2803/scalable-hw-agnostic-inference`` (SD2.1, Flux.1-dev,
Llama-3 / Mistral / DeepSeek-distill LLMs, T5 encoders, DistilBERT, ViT, YOLOS
behind the same FastAPI endpoints), re-designed for one 8x MI355X node:
hand-written gfx950 HIP kernels (``csrc/kernels``), RCCL + xGMI peer-to-peer
collectives for tensor parallelism, and a local router / supervisor /
autoscaler in place of ALB + KEDA + Karpenter.

Subpackages: ``ops`` (kernel wrappers + fp32 torch references), ``parallel``
(process groups, TP layers, collectives), ``models``, ``schedulers``,
``engines`` (diffusion / LLM / encoder engines), ``serving`` (FastAPI apps),
``router``, ``supervisor``, ``autoscaler``, ``controller``, ``bench``, ``ui``,
``weights``, ``tokenizers``, ``utils``, ``runtime`` (native C++ runtime bindings).
"""
__version__ = "0.1.0"
