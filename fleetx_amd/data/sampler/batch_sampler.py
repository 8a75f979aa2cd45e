"""Distributed batch samplers.

Parity: reference ``ppfleetx/data/sampler/batch_sampler.py:31-188``
(``GPTBatchSampler``: contiguous global batches of ``batch_size * nranks``,
each data rank takes its slice, ``consumed_samples`` resume) and Paddle's
``DistributedBatchSampler`` (per-rank interleaved subset, optional shuffle by
epoch).  Here ``consumed_samples`` IS wired to checkpoint resume (reference
defect §2.12 #10): the engine seeks the sampler instead of re-reading and
discarding batches.
"""
import math

import numpy as np

from ...utils import env


class GPTBatchSampler:
    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False,
                 drop_last=False, consumed_samples=0, **kwargs):
        assert isinstance(batch_size, int) and batch_size > 0
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.nranks = num_replicas if num_replicas is not None else env.get_data_world_size()
        self.local_rank = rank if rank is not None else env.get_data_world_rank()
        self.epoch = 0
        self.consumed_samples = consumed_samples
        self.num_samples = int(math.ceil(len(dataset) * 1.0 / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def get_start_end_idx(self):
        s = self.local_rank * self.batch_size
        return s, s + self.batch_size

    def __iter__(self):
        assert self.consumed_samples % self.nranks == 0, \
            "consumed_samples {} must be divisible by nranks {}".format(self.consumed_samples,
                                                                        self.nranks)
        gbs = self.batch_size * self.nranks
        s, e = self.get_start_end_idx()
        batch = []
        for idx in range(self.consumed_samples, self.total_size):
            batch.append(idx % len(self.dataset))
            if len(batch) == gbs:
                yield batch[s:e]
                batch = []
        if not self.drop_last and batch:
            yield batch[s:e] if len(batch) > s else batch

    def __len__(self):
        n = self.num_samples + int(not self.drop_last) * (self.batch_size - 1)
        return n // self.batch_size

    def set_epoch(self, epoch=0, consumed_samples=0):
        self.epoch = epoch
        self.consumed_samples = consumed_samples


class DistributedBatchSampler:
    """Rank ``r`` of ``n`` takes indices ``r, r+n, ...`` (after an optional
    epoch-seeded shuffle), grouped into batches of ``batch_size``."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False,
                 drop_last=False, consumed_samples=0, **kwargs):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.nranks = num_replicas if num_replicas is not None else env.get_data_world_size()
        self.local_rank = rank if rank is not None else env.get_data_world_rank()
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) * 1.0 / self.nranks))
        self.total_size = self.num_samples * self.nranks
        self.consumed_samples = consumed_samples

    def __iter__(self):
        n = len(self.dataset)
        if self.shuffle:
            indices = np.random.RandomState(self.epoch).permutation(n).tolist()
        else:
            indices = list(range(n))
        indices += indices[:(self.total_size - len(indices))]
        mine = indices[self.local_rank:self.total_size:self.nranks]
        skip = self.consumed_samples // self.nranks
        mine = mine[skip:]
        batch = []
        for idx in mine:
            batch.append(idx)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if not self.drop_last and batch:
            yield batch

    def __len__(self):
        n = self.num_samples + int(not self.drop_last) * (self.batch_size - 1)
        return n // self.batch_size

    def set_epoch(self, epoch=0, consumed_samples=0):
        self.epoch = epoch
        self.consumed_samples = consumed_samples
