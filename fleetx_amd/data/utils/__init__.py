"""Collate-function registry."""
from .collate import (collate_fn, gpt_collate_fn, gpt_inference_collate_fn,  # noqa: F401
                      gpt_eval_collate_fn, imagen_collate_fn)

COLLATE_FNS = {
    "collate_fn": collate_fn,
    "gpt_collate_fn": gpt_collate_fn,
    "gpt_inference_collate_fn": gpt_inference_collate_fn,
    "gpt_eval_collate_fn": gpt_eval_collate_fn,
    "imagen_collate_fn": imagen_collate_fn,
}
