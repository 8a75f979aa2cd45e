"""Batchify combinators and the named collate functions.

Parity: reference ``ppfleetx/data/sampler/collate.py:27-317`` (``Stack``,
``Pad``, ``Tuple``, ``Dict``) and ``data/utils/batch_collate_fn.py:30-131``
(``collate_fn``, ``gpt_collate_fn``, ``gpt_inference_collate_fn``,
``gpt_eval_collate_fn``, ``imagen_collate_fn``).  Outputs are torch tensors.
"""
import numbers

import numpy as np
import torch


class Stack:
    def __init__(self, axis=0, dtype=None):
        self.axis, self.dtype = axis, dtype

    def __call__(self, data):
        arr = np.stack(data, axis=self.axis)
        return arr.astype(self.dtype) if self.dtype else arr


class Pad:
    def __init__(self, pad_val=0, axis=0, ret_length=None, dtype=None, pad_right=True):
        self.pad_val, self.axis, self.ret_length = pad_val, axis, ret_length
        self.dtype, self.pad_right = dtype, pad_right

    def __call__(self, data):
        arrs = [np.asarray(d) for d in data]
        lengths = [a.shape[self.axis] for a in arrs]
        maxlen = max(lengths)
        shape = list(arrs[0].shape)
        shape[self.axis] = maxlen
        out = np.full([len(arrs)] + shape, self.pad_val, dtype=self.dtype or arrs[0].dtype)
        for i, a in enumerate(arrs):
            sl = [slice(None)] * a.ndim
            if self.pad_right:
                sl[self.axis] = slice(0, a.shape[self.axis])
            else:
                sl[self.axis] = slice(maxlen - a.shape[self.axis], maxlen)
            out[i][tuple(sl)] = a
        if self.ret_length:
            return out, np.asarray(lengths, dtype=self.ret_length if isinstance(self.ret_length, type) else np.int64)
        return out


class Tuple:
    def __init__(self, fn, *args):
        self.fns = list(fn) if isinstance(fn, (list, tuple)) else [fn] + list(args)

    def __call__(self, data):
        assert len(data[0]) == len(self.fns), "number of fields != number of batchify fns"
        out = []
        for i, f in enumerate(self.fns):
            r = f([x[i] for x in data])
            if isinstance(r, (tuple, list)):
                out.extend(r)
            else:
                out.append(r)
        return tuple(out)


class Dict:
    def __init__(self, fn):
        self.fns = fn

    def __call__(self, data):
        out = []
        for k, f in self.fns.items():
            r = f([x[k] for x in data])
            if isinstance(r, (tuple, list)):
                out.extend(r)
            else:
                out.append(r)
        return tuple(out)


def _to_tensor(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, (list, tuple)):
        return type(x)(_to_tensor(v) for v in x)
    return x


def collate_fn(batch):
    """Generic nested collate: numpy arrays / numbers / dicts / sequences."""
    sample = batch[0]
    if isinstance(sample, np.ndarray):
        return torch.from_numpy(np.stack(batch, axis=0))
    if isinstance(sample, torch.Tensor):
        return torch.stack(batch, 0)
    if isinstance(sample, numbers.Number):
        return torch.as_tensor(np.asarray(batch))
    if isinstance(sample, (str, bytes)):
        return batch
    if isinstance(sample, dict):
        return {k: collate_fn([d[k] for d in batch]) for k in sample}
    if isinstance(sample, (list, tuple)):
        return [collate_fn(list(f)) for f in zip(*batch)]
    raise TypeError("batch data can only contain numpy arrays, numbers, dicts or lists")


def gpt_collate_fn(batch):
    return _to_tensor(list(Tuple([Stack() for _ in batch[0]])(batch)))


def gpt_inference_collate_fn(batch):
    return _to_tensor(list(Tuple(Stack(), Stack())(batch)))


def gpt_eval_collate_fn(batch):
    return _to_tensor(list(Tuple([Stack() for _ in range(6)])(batch)))


def imagen_collate_fn(batch):
    """(image, text_embed [L,D], text_mask [L]) -> padded to the longest text."""
    images = np.stack([b[0] for b in batch])
    maxlen = max(b[1].shape[0] for b in batch)
    dim = batch[0][1].shape[1]
    emb = np.zeros((len(batch), maxlen, dim), dtype=np.float32)
    mask = np.zeros((len(batch), maxlen), dtype=bool)
    for i, b in enumerate(batch):
        n = b[1].shape[0]
        emb[i, :n] = b[1]
        mask[i, :n] = b[2][:n].astype(bool)
    return [torch.from_numpy(images), torch.from_numpy(emb), torch.from_numpy(mask)]
