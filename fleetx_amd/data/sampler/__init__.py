"""Sampler registry."""
from .batch_sampler import GPTBatchSampler, DistributedBatchSampler  # noqa: F401
from ..utils.collate import Stack, Pad, Tuple, Dict  # noqa: F401

SAMPLERS = {"GPTBatchSampler": GPTBatchSampler, "DistributedBatchSampler": DistributedBatchSampler}
