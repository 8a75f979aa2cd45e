"""ERNIE / BERT sentence-pair pretraining samples.

Parity: the reference keeps ``ErnieDataset`` as an import-only stub and
trains ERNIE on GPT-format samples (``ppfleetx/data/dataset/ernie_dataset.py``,
``configs/nlp/ernie/pretrain_ernie_base.yaml:37-50``).  This is
the real thing on the native N-1 builder it was meant for:

* input: the ``_ids.npy`` / ``_idx.npz`` pair written by
  ``data_tools/gpt/preprocess_data.py --split_sentences`` (``lens`` = tokens
  per sentence, ``docs`` = cumulative sentence count per document);
* sample map: ``_native.build_mapping`` (BERT-style packing of whole
  sentences into ``max_seq_len - 3`` tokens with short-sequence sampling,
  mt19937 / mt19937_64 exactly as ``fast_index_map_helpers.cpp``), rows
  ``(first sentence, end sentence, target length)``;
* ``__getitem__``: split the sentences at a random point into segments A / B;
  with probability 1/2 B comes from a random other document
  (``next_sentence_label = 1``); truncate the pair to the target length;
  emit ``[CLS] A [SEP] B [SEP]`` padded to ``max_seq_len``.  Per-sample
  randomness is seeded by ``(seed, index)``, so resume / any worker count
  sees identical samples.  Masked-LM masking is applied on the device by
  :class:`ErnieModule` (dynamic masking).
"""
import os

import numpy as np
import torch

from .gpt_dataset import MODE_TO_INDEX, get_train_data_file, get_train_valid_test_split_


def _truncate_pair(a, b, max_tokens, rng):
    while len(a) + len(b) > max_tokens:
        longer = a if len(a) > len(b) else b
        if rng.random_sample() < 0.5:
            del longer[0]
        else:
            longer.pop()


class ErnieDataset(torch.utils.data.Dataset):
    def __init__(self, input_dir, split, max_seq_len, num_samples, mode, seed=1234, cls_id=1,
                 sep_id=2, pad_id=0, short_seq_prob=0.1, min_num_sent=2, **kwargs):
        files = get_train_data_file(input_dir) if os.path.isdir(input_dir) else [input_dir]
        prefix = files[0]
        self.ids = np.load(prefix + "_ids.npy", mmap_mode="r")
        idx = np.load(prefix + "_idx.npz")
        self.sizes = idx["lens"].astype(np.int32)
        docs = idx["docs"].astype(np.int64)
        ndocs = len(docs) - 1
        bounds = get_train_valid_test_split_(split, ndocs)
        lo, hi = bounds[MODE_TO_INDEX[mode]], bounds[MODE_TO_INDEX[mode] + 1]
        self.docs = docs[lo:hi + 1]
        self.start = np.concatenate([[0], np.cumsum(self.sizes, dtype=np.int64)])
        self.max_seq_len = int(max_seq_len)
        self.cls_id, self.sep_id, self.pad_id = cls_id, sep_id, pad_id
        self.seed = int(seed)
        from ..._C import _native
        self.mapping = _native.build_mapping(self.docs, self.sizes, 1000, int(num_samples),
                                             self.max_seq_len - 3, float(short_seq_prob),
                                             self.seed, False, int(min_num_sent))
        # sentence -> document (for "random next segment" sampling)
        self.nd = len(self.docs) - 1

    def __len__(self):
        return int(self.mapping.shape[0])

    def _sent(self, i):
        return self.ids[self.start[i]:self.start[i + 1]].tolist()

    def __getitem__(self, index):
        s0, s1, target = (int(x) for x in self.mapping[index])
        rng = np.random.RandomState((self.seed * 1000003 + index) % (2 ** 32))
        sents = [self._sent(i) for i in range(s0, s1)]
        a_end = rng.randint(1, len(sents)) if len(sents) > 1 else 1
        a = [t for s in sents[:a_end] for t in s]
        nsp = 0
        if len(sents) == 1 or rng.random_sample() < 0.5:
            nsp = 1  # B from another document
            cur_doc = int(np.searchsorted(self.docs, s0, side="right")) - 1
            d = rng.randint(0, self.nd)
            if self.nd > 1 and d == cur_doc:
                d = (d + 1) % self.nd
            first = int(self.docs[d]) + rng.randint(0, max(1, int(self.docs[d + 1] - self.docs[d])))
            b, i = [], first
            while len(b) < target - len(a) and i < int(self.docs[d + 1]):
                b += self._sent(i)
                i += 1
        else:
            b = [t for s in sents[a_end:] for t in s]
        _truncate_pair(a, b, target, rng)
        toks = [self.cls_id] + a + [self.sep_id] + b + [self.sep_id]
        types = [0] * (len(a) + 2) + [1] * (len(b) + 1)
        n = len(toks)
        out = np.full(self.max_seq_len, self.pad_id, dtype=np.int64)
        tt = np.zeros(self.max_seq_len, dtype=np.int64)
        out[:n] = toks
        tt[:n] = types
        return [out, tt, np.int64(nsp), np.int64(n)]
