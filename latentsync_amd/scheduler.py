"""DDIMScheduler -- the ``scheduler`` object of LipsyncPipeline
(lipsync_pipeline.py:424, 478, 544, 562; scripts/inference.py:40 loads
configs/scheduler_config.json through diffusers).

diffusers 0.32.2 restated: scaled_linear
betas in fp32, alphas_cumprod = cumprod(1 - beta), "leading" timestep spacing
with steps_offset, eta = 0 deterministic update, epsilon prediction, no
clipping / thresholding.  The integer timestep and alpha-bar index math is
exact (checked bit-for-bit against SURVEY.md's known answers).  The window
engine does not call ``step``: it uploads ``coef_table`` once and the fused
HIP kernel ls_ddim_cfg_step applies the same update on device.
"""
import json
import os
from dataclasses import dataclass

import numpy as np
import torch


class _Config(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


@dataclass
class DDIMSchedulerOutput:
    prev_sample: torch.Tensor
    pred_original_sample: torch.Tensor = None


class DDIMScheduler:
    order = 1

    def __init__(self, num_train_timesteps=1000, beta_start=0.0001, beta_end=0.02, beta_schedule="linear",
                 trained_betas=None, clip_sample=True, set_alpha_to_one=True, steps_offset=0,
                 prediction_type="epsilon", timestep_spacing="leading", **unused):
        if beta_schedule == "scaled_linear":
            betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        elif beta_schedule == "linear":
            betas = torch.linspace(beta_start, beta_end, num_train_timesteps, dtype=torch.float32)
        elif trained_betas is not None:
            betas = torch.tensor(trained_betas, dtype=torch.float32)
        else:
            raise NotImplementedError(beta_schedule)
        if prediction_type != "epsilon" or timestep_spacing != "leading":
            raise NotImplementedError("only the epsilon / leading DDIM configuration is on the LatentSync path")
        self._internal_dict = _Config(num_train_timesteps=num_train_timesteps, beta_start=beta_start,
                                      beta_end=beta_end, beta_schedule=beta_schedule, clip_sample=clip_sample,
                                      set_alpha_to_one=set_alpha_to_one, steps_offset=steps_offset,
                                      prediction_type=prediction_type, timestep_spacing=timestep_spacing)
        self.betas = betas
        self.alphas = 1.0 - betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.init_noise_sigma = 1.0
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, num_train_timesteps)[::-1].copy().astype(np.int64))

    @property
    def config(self):
        return self._internal_dict

    @classmethod
    def from_config(cls, config):
        return cls(**{k: v for k, v in dict(config).items() if not k.startswith("_")})

    @classmethod
    def from_pretrained(cls, path, subfolder=None, **kw):
        """Directory holding scheduler_config.json (e.g. the reference's ``configs``)."""
        d = os.path.join(path, subfolder) if subfolder else path
        f = d if d.endswith(".json") else os.path.join(d, "scheduler_config.json")
        with open(f) as fh:
            return cls.from_config(json.load(fh))

    def set_timesteps(self, num_inference_steps, device=None):
        T = self.config.num_train_timesteps
        if num_inference_steps > T:
            raise ValueError(f"num_inference_steps {num_inference_steps} > num_train_timesteps {T}")
        self.num_inference_steps = num_inference_steps
        ratio = T // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
        ts += self.config.steps_offset
        self.timesteps = torch.from_numpy(ts).to(device)

    def scale_model_input(self, sample, timestep=None):
        return sample

    def _alphas(self, t):
        prev = int(t) - self.config.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[int(t)]
        a_p = self.alphas_cumprod[prev] if prev >= 0 else self.final_alpha_cumprod
        return a_t, a_p

    def step(self, model_output, timestep, sample, eta=0.0, use_clipped_model_output=False, generator=None,
             variance_noise=None, return_dict=True):
        if self.num_inference_steps is None:
            raise ValueError("Number of inference steps is 'None', you need to run 'set_timesteps' first")
        if eta != 0.0:
            raise NotImplementedError("eta > 0 (stochastic DDIM) is not used by LatentSync inference")
        a_t, a_p = self._alphas(timestep)
        x0 = (sample - (1 - a_t) ** 0.5 * model_output) / a_t ** 0.5
        prev = a_p ** 0.5 * x0 + (1 - a_p) ** 0.5 * model_output
        if not return_dict:
            return (prev,)
        return DDIMSchedulerOutput(prev_sample=prev, pred_original_sample=x0)

    def coef_table(self, device=None):
        """fp32 [n_steps][4] = sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev) in
        timestep order -- consumed by ls_ddim_cfg_step."""
        rows = []
        for t in self.timesteps.tolist():
            a_t, a_p = self._alphas(t)
            rows.append([float(a_t ** 0.5), float((1 - a_t) ** 0.5), float(a_p ** 0.5), float((1 - a_p) ** 0.5)])
        return torch.tensor(rows, dtype=torch.float32, device=device)
