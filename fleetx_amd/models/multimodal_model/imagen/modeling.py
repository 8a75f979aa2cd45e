"""Cascaded text-to-image diffusion (Imagen): training losses and sampling.

Parity: reference ``models/multimodal_model/imagen/modeling.py:89-823`` (C35):
``ImagenCriterion`` (l1 / mse / smooth-l1 with p2 reweighting
``(k + exp(log_snr)) ** -gamma``), ``ImagenModel`` (per-U-Net noise schedules
and objectives, low-resolution conditioning with noise augmentation,
classifier-free-guidance dropout, ``p_losses`` / ``forward`` for training,
``p_mean_variance`` with dynamic thresholding, ``p_sample``, ``p_sample_loop``
with inpainting and ``sample`` across the cascade) and the model builders.

Differences: ``random_crop_sizes`` is implemented (the reference calls an
undefined kornia ``K``), and ``imagen_SR64to1024`` is omitted (the reference
references an undefined class).  The diffusion math runs in fp32; only the
U-Net runs in the compute dtype.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .diffusion import (GaussianDiffusionContinuousTimes, cast_tuple, cast_uint8_images_to_float,
                        default, exists, normalize_neg_one_to_one, pad_tuple_to_length,
                        resize_image_to, right_pad_dims_to, unnormalize_zero_to_one)
from .unet import Unet, Unet64_397M, BaseUnet64, SRUnet256, SRUnet1024


class ImagenCriterion(nn.Module):
    def __init__(self, name="mse_loss", p2_loss_weight_k=1.0):
        super().__init__()
        self.p2_loss_weight_k = p2_loss_weight_k
        fns = {"l1_loss": F.l1_loss, "mse_loss": F.mse_loss, "smooth_l1_loss": F.smooth_l1_loss}
        if name not in fns:
            raise NotImplementedError(name)
        self.loss_func = fns[name]

    def forward(self, pred, target, log_snr, p2_loss_weight_gamma):
        losses = self.loss_func(pred.float(), target.float(), reduction="none")
        losses = losses.reshape(losses.shape[0], -1).mean(-1)
        if p2_loss_weight_gamma > 0:
            losses = losses * (self.p2_loss_weight_k + log_snr.float().exp()) ** -p2_loss_weight_gamma
        return losses.mean()


def _random_crop(size, *tensors):
    h, w = tensors[0].shape[-2:]
    i = int(torch.randint(0, h - size + 1, (1,)))
    j = int(torch.randint(0, w - size + 1, (1,)))
    return [None if t is None else t[..., i:i + size, j:j + size] for t in tensors]


class ImagenModel(nn.Module):
    def __init__(self, unets, image_sizes, text_encoder_name="t5/t5-11b", text_embed_dim=1024,
                 in_chans=3, timesteps=1000, cond_drop_prob=0.1, num_classes=None,
                 noise_schedules="cosine", pred_objectives="noise", random_crop_sizes=None,
                 lowres_noise_schedule="linear", lowres_sample_noise_level=0.2,
                 per_sample_random_aug_noise_level=False, condition_on_text=True,
                 auto_normalize_img=True, p2_loss_weight_gamma=0.5, dynamic_thresholding=True,
                 dynamic_thresholding_percentile=0.95, only_train_unet_number=None,
                 use_recompute=False, fused_linear=False, **kwargs):
        super().__init__()
        self.condition_on_text = condition_on_text
        self.unconditional = not condition_on_text
        self.channels = in_chans
        unets = cast_tuple(unets)
        n = len(unets)
        timesteps = cast_tuple(timesteps, n)
        schedules = pad_tuple_to_length(cast_tuple(noise_schedules), 2, "cosine")
        schedules = pad_tuple_to_length(schedules, n, "linear")
        self.noise_schedulers = [GaussianDiffusionContinuousTimes(noise_schedule=s, timesteps=t)
                                 for t, s in zip(timesteps, schedules)]
        self.random_crop_sizes = cast_tuple(random_crop_sizes, n)
        assert not exists(self.random_crop_sizes[0]), "base unet must not be randomly cropped"
        self.lowres_noise_schedule = GaussianDiffusionContinuousTimes(
            noise_schedule=lowres_noise_schedule)
        self.pred_objectives = cast_tuple(pred_objectives, n)
        self.text_encoder_name = text_encoder_name
        self.text_embed_dim = default(text_embed_dim, 1024)
        self.only_train_unet_number = only_train_unet_number
        ulist = []
        for ind, u in enumerate(unets):
            assert isinstance(u, Unet)
            u = u.cast_model_parameters(
                lowres_cond=ind > 0, cond_on_text=condition_on_text,
                text_embed_dim=self.text_embed_dim if condition_on_text else None,
                channels=in_chans, channels_out=in_chans)
            u.use_recompute = use_recompute
            ulist.append(u)
        self.unets = nn.ModuleList(ulist)
        self.image_sizes = cast_tuple(image_sizes)
        assert n == len(self.image_sizes)
        self.sample_channels = cast_tuple(in_chans, n)
        assert tuple(u.lowres_cond for u in self.unets) == (False, *((True,) * (n - 1)))
        self.lowres_sample_noise_level = lowres_sample_noise_level
        self.per_sample_random_aug_noise_level = per_sample_random_aug_noise_level
        self.cond_drop_prob = cond_drop_prob
        self.can_classifier_guidance = cond_drop_prob > 0.0
        self.normalize_img = normalize_neg_one_to_one if auto_normalize_img else (lambda t: t)
        self.unnormalize_img = unnormalize_zero_to_one if auto_normalize_img else (lambda t: t)
        self.input_image_range = (0.0 if auto_normalize_img else -1.0, 1.0)
        if isinstance(dynamic_thresholding, str):  # the reference YAMLs write "True,"
            dynamic_thresholding = dynamic_thresholding.strip().rstrip(",").lower() == "true"
        self.dynamic_thresholding = cast_tuple(dynamic_thresholding, n)
        self.dynamic_thresholding_percentile = dynamic_thresholding_percentile
        self.p2_loss_weight_gamma = cast_tuple(p2_loss_weight_gamma, n)
        assert all(g <= 2 for g in self.p2_loss_weight_gamma)

    def get_unet(self, unet_number):
        assert 0 < unet_number <= len(self.unets)
        return self.unets[unet_number - 1]

    # ---------------------------------------------------------------- sampling
    def p_mean_variance(self, unet, x, t, *, noise_scheduler, text_embeds=None, text_mask=None,
                        cond_images=None, lowres_cond_img=None, lowres_noise_times=None,
                        cond_scale=1.0, model_output=None, t_next=None, pred_objective="noise",
                        dynamic_threshold=True):
        assert not (cond_scale != 1.0 and not self.can_classifier_guidance)
        pred = model_output
        if pred is None:
            pred = unet.forward_with_cond_scale(
                x, noise_scheduler.get_condition(t), text_embeds=text_embeds, text_mask=text_mask,
                cond_images=cond_images, cond_scale=cond_scale, lowres_cond_img=lowres_cond_img,
                lowres_noise_times=self.lowres_noise_schedule.get_condition(lowres_noise_times))
        pred = pred.float()
        if pred_objective == "noise":
            x_start = noise_scheduler.predict_start_from_noise(x, t=t, noise=pred)
        elif pred_objective == "x_start":
            x_start = pred
        else:
            raise ValueError("unknown objective {}".format(pred_objective))
        if dynamic_threshold:
            s = torch.quantile(x_start.reshape(x_start.shape[0], -1).abs(),
                               self.dynamic_thresholding_percentile, dim=-1)
            s = right_pad_dims_to(x_start, s.clamp(min=1.0))
            x_start = x_start.clamp(-s, s) / s
        else:
            x_start = x_start.clamp(-1.0, 1.0)
        return noise_scheduler.q_posterior(x_start=x_start, x_t=x, t=t, t_next=t_next), x_start

    @torch.no_grad()
    def p_sample(self, unet, x, t, *, noise_scheduler, t_next=None, **kw):
        (mean, _, log_var), x_start = self.p_mean_variance(unet, x, t, t_next=t_next,
                                                           noise_scheduler=noise_scheduler, **kw)
        noise = torch.randn_like(x)
        last = (t_next == 0).float()
        nonzero = right_pad_dims_to(x, 1 - last)
        return mean + nonzero * (0.5 * log_var).exp() * noise, x_start

    @torch.no_grad()
    def p_sample_loop(self, unet, shape, *, noise_scheduler, lowres_cond_img=None,
                      lowres_noise_times=None, text_embeds=None, text_mask=None, cond_images=None,
                      inpaint_images=None, inpaint_masks=None, inpaint_resample_times=5,
                      init_images=None, skip_steps=None, cond_scale=1, pred_objective="noise",
                      dynamic_threshold=True, device=None):
        b = shape[0]
        img = torch.randn(shape, device=device)
        if exists(init_images):
            img = img + init_images
        has_inpaint = exists(inpaint_images) and exists(inpaint_masks)
        resample_times = inpaint_resample_times if has_inpaint else 1
        if has_inpaint:
            inpaint_images = resize_image_to(self.normalize_img(inpaint_images), shape[-1])
            inpaint_masks = resize_image_to(inpaint_masks[:, None].float(), shape[-1]).bool()
        steps = noise_scheduler.get_sampling_timesteps(b, device=device)[default(skip_steps, 0):]
        for times, times_next in steps:
            is_last = times_next == 0
            for r in reversed(range(resample_times)):
                if has_inpaint:
                    noised, _ = noise_scheduler.q_sample(inpaint_images, t=times)
                    img = img * ~inpaint_masks + noised * inpaint_masks
                img, _ = self.p_sample(unet, img, times, t_next=times_next,
                                       noise_scheduler=noise_scheduler, text_embeds=text_embeds,
                                       text_mask=text_mask, cond_images=cond_images,
                                       cond_scale=cond_scale, lowres_cond_img=lowres_cond_img,
                                       lowres_noise_times=lowres_noise_times,
                                       pred_objective=pred_objective,
                                       dynamic_threshold=dynamic_threshold)
                if has_inpaint and not (r == 0 or bool(is_last.all())):
                    renoised = noise_scheduler.q_sample_from_to(img, times_next, times)
                    img = torch.where(right_pad_dims_to(img, is_last), img, renoised)
        img = img.clamp(-1.0, 1.0)
        if has_inpaint:
            img = img * ~inpaint_masks + inpaint_images * inpaint_masks
        return self.unnormalize_img(img)

    @torch.no_grad()
    def sample(self, texts=None, text_masks=None, text_embeds=None, cond_images=None,
               inpaint_images=None, inpaint_masks=None, inpaint_resample_times=5,
               init_images=None, skip_steps=None, batch_size=1, cond_scale=1.0,
               lowres_sample_noise_level=None, stop_at_unet_number=None,
               return_all_unet_outputs=False, return_pil_images=False):
        was_training = self.training
        self.eval()
        device = next(self.parameters()).device
        cond_images = cast_uint8_images_to_float(cond_images)
        if not self.unconditional:
            assert exists(text_embeds), "text embeddings must be passed in"
            assert text_embeds.shape[-1] == self.text_embed_dim
            text_masks = default(text_masks, lambda: (text_embeds != 0.0).any(-1))
            batch_size = text_embeds.shape[0]
        assert not (exists(inpaint_images) ^ exists(inpaint_masks))
        outputs = []
        level = default(lowres_sample_noise_level, self.lowres_sample_noise_level)
        n = len(self.unets)
        cond_scale = cast_tuple(cond_scale, n)
        init_images = [self.normalize_img(i) if exists(i) else None
                       for i in cast_tuple(init_images, n)]
        skip_steps = cast_tuple(skip_steps, n)
        img = None
        for num, unet, ch, size, sched, obj, dyn, cs, init, skip in zip(
                range(1, n + 1), self.unets, self.sample_channels, self.image_sizes,
                self.noise_schedulers, self.pred_objectives, self.dynamic_thresholding,
                cond_scale, init_images, skip_steps):
            lowres_img = lowres_times = None
            if unet.lowres_cond:
                lowres_times = self.lowres_noise_schedule.get_times(batch_size, level, device)
                lowres_img = self.normalize_img(resize_image_to(img, size))
                lowres_img, _ = self.lowres_noise_schedule.q_sample(lowres_img, t=lowres_times)
            img = self.p_sample_loop(unet, (batch_size, ch, size, size), noise_scheduler=sched,
                                     lowres_cond_img=lowres_img, lowres_noise_times=lowres_times,
                                     text_embeds=text_embeds, text_mask=text_masks,
                                     cond_images=cond_images, inpaint_images=inpaint_images,
                                     inpaint_masks=inpaint_masks,
                                     inpaint_resample_times=inpaint_resample_times,
                                     init_images=init, skip_steps=skip, cond_scale=cs,
                                     pred_objective=obj, dynamic_threshold=dyn, device=device)
            outputs.append(img)
            if exists(stop_at_unet_number) and stop_at_unet_number == num:
                break
        self.train(was_training)
        outs = outputs if return_all_unet_outputs else outputs[-1:]
        if return_pil_images:
            from PIL import Image
            pil = [[Image.fromarray((im.permute(1, 2, 0).clamp(0, 1) * 255).byte().cpu().numpy())
                    for im in o] for o in outs]
            return pil if return_all_unet_outputs else pil[0]
        return outs if return_all_unet_outputs else outs[0]

    # ---------------------------------------------------------------- training
    def p_losses(self, unet, x_start, times, *, noise_scheduler, lowres_cond_img=None,
                 lowres_aug_times=None, text_embeds=None, text_mask=None, cond_images=None,
                 noise=None, pred_objective="noise", p2_loss_weight_gamma=0.0,
                 random_crop_size=None):
        x_start = self.normalize_img(x_start.float())
        noise = default(noise, lambda: torch.randn_like(x_start))
        if exists(lowres_cond_img):
            lowres_cond_img = self.normalize_img(lowres_cond_img.float())
        if exists(random_crop_size):
            x_start, lowres_cond_img, noise = _random_crop(random_crop_size, x_start,
                                                           lowres_cond_img, noise)
        x_noisy, log_snr = noise_scheduler.q_sample(x_start=x_start, t=times, noise=noise)
        lowres_noisy = None
        if exists(lowres_cond_img):
            lowres_aug_times = default(lowres_aug_times, times)
            lowres_noisy, _ = self.lowres_noise_schedule.q_sample(lowres_cond_img,
                                                                  t=lowres_aug_times)
        pred = unet(x_noisy, noise_scheduler.get_condition(times), text_embeds=text_embeds,
                    text_mask=text_mask, cond_images=cond_images,
                    lowres_noise_times=self.lowres_noise_schedule.get_condition(lowres_aug_times),
                    lowres_cond_img=lowres_noisy, cond_drop_prob=self.cond_drop_prob)
        if pred_objective == "noise":
            target = noise
        elif pred_objective == "x_start":
            target = x_start
        else:
            raise ValueError("unknown objective {}".format(pred_objective))
        return pred, target, log_snr, p2_loss_weight_gamma

    def forward(self, images, unet=None, texts=None, text_embeds=None, text_masks=None,
                unet_number=None, cond_images=None):
        assert images.shape[-1] == images.shape[-2], "images must be square"
        assert not (len(self.unets) > 1 and not exists(unet_number)), \
            "specify which unet to train for a cascade"
        unet_number = default(unet_number, 1)
        assert not exists(self.only_train_unet_number) or self.only_train_unet_number == unet_number
        images = cast_uint8_images_to_float(images)
        cond_images = cast_uint8_images_to_float(cond_images)
        idx = unet_number - 1
        unet = default(unet, lambda: self.get_unet(unet_number))
        sched = self.noise_schedulers[idx]
        target_size = self.image_sizes[idx]
        prev_size = self.image_sizes[idx - 1] if idx > 0 else None
        b, c, h, w = images.shape
        dev = images.device
        assert c == self.channels and h >= target_size
        times = sched.sample_random_times(b, device=dev)
        if not self.unconditional:
            assert exists(text_embeds), "text embeddings must be passed in"
            assert text_embeds.shape[-1] == self.text_embed_dim
            text_masks = default(text_masks, lambda: (text_embeds != 0.0).any(-1))
        lowres_img = lowres_times = None
        if exists(prev_size):
            lowres_img = resize_image_to(images, prev_size, clamp_range=self.input_image_range)
            lowres_img = resize_image_to(lowres_img, target_size, clamp_range=self.input_image_range)
            if self.per_sample_random_aug_noise_level:
                lowres_times = self.lowres_noise_schedule.sample_random_times(b, device=dev)
            else:
                lowres_times = self.lowres_noise_schedule.sample_random_times(1, device=dev).expand(b)
        images = resize_image_to(images, target_size)
        return self.p_losses(unet, images, times, text_embeds=text_embeds, text_mask=text_masks,
                             cond_images=cond_images, noise_scheduler=sched,
                             lowres_cond_img=lowres_img, lowres_aug_times=lowres_times,
                             pred_objective=self.pred_objectives[idx],
                             p2_loss_weight_gamma=self.p2_loss_weight_gamma[idx],
                             random_crop_size=self.random_crop_sizes[idx])


def _u(preset, unet_kwargs):
    return preset(**dict(unet_kwargs or {}))


# ``unet_kwargs`` (optional, from ``Model.unet_kwargs``) overrides preset U-Net
# hyper-parameters, e.g. a narrow U-Net for smoke tests.
def imagen_397M_text2im_64(unet_kwargs=None, **kw):
    return ImagenModel(unets=_u(Unet64_397M, unet_kwargs), image_sizes=(64,), **kw)


def imagen_2B_text2im_64(unet_kwargs=None, **kw):
    return ImagenModel(unets=_u(BaseUnet64, unet_kwargs), image_sizes=(64,), **kw)


def imagen_text2im_64_SR256(unet_kwargs=None, **kw):
    return ImagenModel(unets=(_u(BaseUnet64, unet_kwargs), _u(SRUnet256, unet_kwargs)),
                       image_sizes=(64, 256), **kw)


def imagen_SR256(unet_kwargs=None, **kw):
    return ImagenModel(unets=_u(SRUnet256, unet_kwargs), image_sizes=(256,), **kw)


def imagen_SR512(unet_kwargs=None, **kw):
    return ImagenModel(unets=_u(SRUnet1024, unet_kwargs), image_sizes=(512,), **kw)


def imagen_SR1024(unet_kwargs=None, **kw):
    return ImagenModel(unets=_u(SRUnet1024, unet_kwargs), image_sizes=(1024,), **kw)


BUILDERS = {f.__name__: f for f in (imagen_397M_text2im_64, imagen_2B_text2im_64,
                                    imagen_text2im_64_SR256, imagen_SR256, imagen_SR512,
                                    imagen_SR1024)}
