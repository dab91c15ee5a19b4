# MI355X serving image (replaces the reference's per-accelerator CUDA / Neuron / Graviton images,
# serving-container-build/ and app/Dockerfile.template): ROCm + PyTorch-ROCm base, gfx950 kernels built at
# image build time, one image for every model server (the server module is the container command).
FROM rocm/pytorch:latest
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /opt/shai
COPY . /opt/shai
RUN python csrc/build.py && pip install --no-build-isolation --no-deps .
EXPOSE 8000
# e.g. docker run --device=/dev/kfd --device=/dev/dri -e MODEL_ID=stabilityai/stable-diffusion-2-1 <img> shai-serve-sd
#      docker run ... <img> shai-launch --config /opt/shai/config/node.yaml      (router + supervisor, whole node)
CMD ["shai-serve-sd"]
