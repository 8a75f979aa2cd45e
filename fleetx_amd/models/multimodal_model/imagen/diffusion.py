"""Continuous-time Gaussian diffusion and small helpers for Imagen.

Parity: reference ``models/multimodal_model/imagen/utils.py:26-431`` (C35):
``beta_linear_log_snr`` / ``alpha_cosine_log_snr`` schedules,
``GaussianDiffusionContinuousTimes`` (random times, sampling time pairs,
``q_sample``, ``q_sample_from_to``, ``q_posterior``,
``predict_start_from_noise``), nearest resize, [-1, 1] normalisation.

All schedule math is done in fp32 whatever the U-Net dtype is.  The
reference's ``q_sample_from_to`` evaluates the destination log-SNR at the
*source* time (``utils.py:409``); here it uses the destination time.
"""
import math

import torch
import torch.nn.functional as F


def exists(v):
    return v is not None


def default(v, d):
    if exists(v):
        return v
    return d() if callable(d) else d


def cast_tuple(val, length=None):
    if isinstance(val, list):
        val = tuple(val)
    out = val if isinstance(val, tuple) else ((val,) * (length or 1))
    if exists(length):
        assert len(out) == length, "expected length {} got {}".format(length, len(out))
    return out


def pad_tuple_to_length(t, length, fillvalue=None):
    rem = length - len(t)
    return t if rem <= 0 else (*t, *((fillvalue,) * rem))


def right_pad_dims_to(x, t):
    pad = x.ndim - t.ndim
    return t if pad <= 0 else t.reshape(*t.shape, *((1,) * pad))


def resize_image_to(image, size, clamp_range=None):
    if image.shape[-1] == size:
        return image
    out = F.interpolate(image, size=(size, size), mode="nearest")
    return out.clamp(*clamp_range) if exists(clamp_range) else out


def normalize_neg_one_to_one(img):
    return img * 2 - 1


def unnormalize_zero_to_one(img):
    return (img + 1) * 0.5


def cast_uint8_images_to_float(images):
    if images is None or images.dtype != torch.uint8:
        return images
    return images.float() / 255.0


def _log(t, eps=1e-12):
    return torch.log(t.clamp(min=eps))


def beta_linear_log_snr(t):
    return -torch.log(torch.expm1(1e-4 + 10 * t ** 2))


def alpha_cosine_log_snr(t, s=0.008):
    return -_log(torch.cos((t + s) / (1 + s) * math.pi * 0.5) ** -2 - 1, eps=1e-5)


def log_snr_to_alpha_sigma(log_snr):
    return torch.sqrt(torch.sigmoid(log_snr)), torch.sqrt(torch.sigmoid(-log_snr))


class GaussianDiffusionContinuousTimes:
    def __init__(self, *, noise_schedule, timesteps=1000):
        if noise_schedule == "linear":
            self.log_snr = beta_linear_log_snr
        elif noise_schedule == "cosine":
            self.log_snr = alpha_cosine_log_snr
        else:
            raise ValueError("invalid noise schedule {}".format(noise_schedule))
        self.num_timesteps = timesteps

    def get_times(self, batch, noise_level, device=None):
        return torch.full((batch,), float(noise_level), device=device, dtype=torch.float32)

    def sample_random_times(self, batch, max_thres=0.999, device=None):
        return torch.rand(batch, device=device) * max_thres

    def get_condition(self, times):
        return None if times is None else self.log_snr(times.float())

    def get_sampling_timesteps(self, batch, device=None):
        times = torch.linspace(1.0, 0.0, self.num_timesteps + 1, device=device)
        times = times.unsqueeze(0).expand(batch, -1)
        return list(zip(times[:, :-1].unbind(-1), times[:, 1:].unbind(-1)))

    def q_posterior(self, x_start, x_t, t, *, t_next=None):
        t_next = default(t_next, lambda: (t - 1.0 / self.num_timesteps).clamp(min=0.0))
        log_snr = right_pad_dims_to(x_t, self.log_snr(t.float()))
        log_snr_next = right_pad_dims_to(x_t, self.log_snr(t_next.float()))
        alpha, sigma = log_snr_to_alpha_sigma(log_snr)
        alpha_next, sigma_next = log_snr_to_alpha_sigma(log_snr_next)
        c = -torch.expm1(log_snr - log_snr_next)
        mean = alpha_next * (x_t * (1 - c) / alpha + c * x_start)
        var = sigma_next ** 2 * c
        return mean, var, _log(var, eps=1e-20)

    def q_sample(self, x_start, t, noise=None):
        if isinstance(t, float):
            t = torch.full((x_start.shape[0],), t, device=x_start.device)
        noise = default(noise, lambda: torch.randn_like(x_start))
        log_snr = self.log_snr(t.float())
        alpha, sigma = log_snr_to_alpha_sigma(right_pad_dims_to(x_start, log_snr))
        return alpha * x_start + sigma * noise, log_snr

    def q_sample_from_to(self, x_from, from_t, to_t, noise=None):
        b = x_from.shape[0]
        if isinstance(from_t, float):
            from_t = torch.full((b,), from_t, device=x_from.device)
        if isinstance(to_t, float):
            to_t = torch.full((b,), to_t, device=x_from.device)
        noise = default(noise, lambda: torch.randn_like(x_from))
        alpha, sigma = log_snr_to_alpha_sigma(right_pad_dims_to(x_from, self.log_snr(from_t)))
        alpha_to, sigma_to = log_snr_to_alpha_sigma(right_pad_dims_to(x_from, self.log_snr(to_t)))
        return x_from * (alpha_to / alpha) + noise * (sigma_to * alpha - sigma * alpha_to) / alpha

    def predict_start_from_noise(self, x_t, t, noise):
        log_snr = right_pad_dims_to(x_t, self.log_snr(t.float()))
        alpha, sigma = log_snr_to_alpha_sigma(log_snr)
        return (x_t - sigma * noise) / alpha.clamp(min=1e-8)
