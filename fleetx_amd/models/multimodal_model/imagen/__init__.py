"""Imagen cascaded diffusion (reference ``models/multimodal_model/imagen``)."""
from .modeling import (ImagenModel, ImagenCriterion, BUILDERS, imagen_397M_text2im_64,  # noqa: F401
                       imagen_2B_text2im_64, imagen_text2im_64_SR256, imagen_SR256, imagen_SR512,
                       imagen_SR1024)
from .unet import Unet, Unet64_397M, BaseUnet64, SRUnet256, SRUnet1024  # noqa: F401
from .diffusion import GaussianDiffusionContinuousTimes  # noqa: F401
