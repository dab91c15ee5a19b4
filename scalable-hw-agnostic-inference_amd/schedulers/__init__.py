"""Diffusion samplers.  Host side only computes the timestep / alpha tables; the
per-step update (with classifier-free guidance folded in) is one fused kernel
(``ops.sched_step``).

* :class:`DDIMScheduler` -- diffusers DDIMScheduler semantics (eta = 0,
  "leading" spacing, steps_offset=1, set_alpha_to_one=False), epsilon or
  v-prediction.  The reference swaps SD2.1 to DDIM (app/run-sd.py:108).
* :class:`EulerDiscreteScheduler` -- k-diffusion Euler in sigma space.
* :class:`FlowMatchEulerScheduler` -- Flux.1 rectified-flow Euler with the
  resolution-dependent time shift (FlowMatchEulerDiscreteScheduler).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List

import numpy as np

PRED_EPS, PRED_V, PRED_FLOW = 0, 1, 2


@dataclass
class StepParams:
    t: float          # model timestep input
    a_t: float        # alpha_cumprod at t (DDIM)
    a_prev: float     # alpha_cumprod at previous t
    dt: float = 0.0   # flow / euler step size
    scale_in: float = 1.0  # model-input scaling (Euler)


def scaled_linear_alphas(n_train=1000, beta_start=0.00085, beta_end=0.012) -> np.ndarray:
    betas = np.linspace(beta_start ** 0.5, beta_end ** 0.5, n_train, dtype=np.float64) ** 2
    return np.cumprod(1.0 - betas)


class DDIMScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012, prediction_type="v_prediction",
                 steps_offset=1, set_alpha_to_one=False):
        self.n_train = num_train_timesteps
        self.alphas_cumprod = scaled_linear_alphas(num_train_timesteps, beta_start, beta_end)
        self.final_alpha = 1.0 if set_alpha_to_one else float(self.alphas_cumprod[0])
        self.steps_offset = steps_offset
        self.pred_type = PRED_V if prediction_type == "v_prediction" else PRED_EPS
        self.init_noise_sigma = 1.0

    def steps(self, num_inference_steps: int) -> List[StepParams]:
        ratio = self.n_train // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].astype(np.int64) + self.steps_offset
        out = []
        for t in ts:
            prev = t - ratio
            a_t = float(self.alphas_cumprod[t])
            a_prev = float(self.alphas_cumprod[prev]) if prev >= 0 else self.final_alpha
            out.append(StepParams(float(t), a_t, a_prev))
        return out


class EulerDiscreteScheduler:
    """Euler (k-diffusion) for epsilon-prediction models: x <- x + (sigma_next - sigma) * eps.
    Implemented through the fused kernel's flow path on eps (dt = sigma_next - sigma)."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012):
        ac = scaled_linear_alphas(num_train_timesteps, beta_start, beta_end)
        self.sigmas_train = ((1 - ac) / ac) ** 0.5
        self.n_train = num_train_timesteps
        self.pred_type = PRED_FLOW

    def steps(self, num_inference_steps: int) -> List[StepParams]:
        ts = np.linspace(0, self.n_train - 1, num_inference_steps, dtype=np.float64)[::-1]
        sig = np.interp(ts, np.arange(self.n_train), self.sigmas_train)
        sig = np.append(sig, 0.0)
        self.init_noise_sigma = float((sig[0] ** 2 + 1) ** 0.5)
        return [StepParams(float(t), 0.0, 0.0, float(sig[i + 1] - sig[i]), float(1.0 / (sig[i] ** 2 + 1) ** 0.5))
                for i, t in enumerate(ts)]


class FlowMatchEulerScheduler:
    """Flux.1 flow matching: sigmas linear in [1, 1/N], time-shifted by mu(image_seq_len)."""

    def __init__(self, num_train_timesteps=1000, base_shift=0.5, max_shift=1.15, base_seq_len=256,
                 max_seq_len=4096, use_dynamic_shifting=True, shift=3.0):
        self.n_train = num_train_timesteps
        self.base_shift, self.max_shift = base_shift, max_shift
        self.base_seq_len, self.max_seq_len = base_seq_len, max_seq_len
        self.dynamic = use_dynamic_shifting
        self.shift = shift
        self.pred_type = PRED_FLOW
        self.init_noise_sigma = 1.0

    def mu(self, image_seq_len: int) -> float:
        m = (self.max_shift - self.base_shift) / (self.max_seq_len - self.base_seq_len)
        b = self.base_shift - m * self.base_seq_len
        return image_seq_len * m + b

    def steps(self, num_inference_steps: int, image_seq_len: int = 4096) -> List[StepParams]:
        sig = np.linspace(1.0, 1.0 / num_inference_steps, num_inference_steps)
        if self.dynamic:
            mu = self.mu(image_seq_len)
            sig = math.exp(mu) / (math.exp(mu) + (1 / sig - 1))
        else:
            sig = self.shift * sig / (1 + (self.shift - 1) * sig)
        sig = np.append(sig, 0.0)
        return [StepParams(float(sig[i] * self.n_train), 0.0, 0.0, float(sig[i + 1] - sig[i]))
                for i in range(num_inference_steps)]
