"""Megatron-style packed GPT datasets (+ a synthetic one for benchmarks).

Parity: reference ``ppfleetx/data/dataset/gpt_dataset.py:32-627`` (D02/D05):
``<prefix>_ids.npy`` (mmap token stream) + ``<prefix>_idx.npz{lens}``,
train/valid/test document split, doc/sample/shuffle index maps cached next to
the data as ``*_indexmap_*`` ``.npy`` files (built by local rank 0 with the
native ``build_sample_idx``; other ranks wait for the files), samples of
``[tokens, position_ids, labels, loss_mask]`` with ``loss_mask = 0`` on EOS;
``LM_Eval_Dataset`` (WikiText strided windows, detokenizer) and
``Lambada_Eval_Dataset`` (last-word cloze).

Differences: the EOS id is a parameter (default 50256 = GPT-2) instead of
loading a downloaded tokenizer in every worker; index files are written
atomically (tmp + rename) so waiting ranks never read a partial file.
"""
import json
import math
import os
import re
import time

import numpy as np
import torch

from ...utils.log import logger
from ...utils import env

MODE_TO_INDEX = {"Train": 0, "Eval": 1, "Test": 2}


def get_train_data_file(input_dir):
    files = [os.path.join(input_dir, f)[:-len("_idx.npz")] for f in sorted(os.listdir(input_dir))
             if f.endswith("_idx.npz")]
    if not files:
        raise RuntimeError("no xxx_ids.npy / xxx_idx.npz dataset in '{}'".format(input_dir))
    return files


def get_train_valid_test_split_(splits, size):
    splits = [float(s) for s in splits]
    while len(splits) < 3:
        splits.append(0.0)
    splits = splits[:3]
    total = sum(splits)
    assert total > 0.0
    splits = [s / total for s in splits]
    idx = [0]
    for i, s in enumerate(splits):
        idx.append(idx[i] + int(round(s * float(size))))
    diff = idx[-1] - size
    for i in range(1, len(idx)):
        idx[i] -= diff
    assert idx[-1] == size
    return idx


def _num_epochs(tokens_per_epoch, seq_length, num_samples):
    epochs, total = 0, 0
    while True:
        epochs += 1
        total += tokens_per_epoch
        if (total - 1) // seq_length >= num_samples:
            return epochs


def _build_doc_idx(documents, num_epochs, np_rng, separate_last_epoch):
    if not separate_last_epoch or num_epochs == 1:
        doc_idx = np.tile(np.asarray(documents), num_epochs).astype(np.int32)
        return doc_idx
    first = _build_doc_idx(documents, num_epochs - 1, np_rng, False)
    last = _build_doc_idx(documents, 1, np_rng, False)
    return np.concatenate((first, last))


def build_sample_idx_py(sizes, doc_idx, seq_length, num_epochs, tokens_per_epoch):
    """Pure-Python oracle of the native builder (used by tests)."""
    num_samples = (num_epochs * tokens_per_epoch - 1) // seq_length
    out = np.zeros([int(num_samples) + 1, 2], dtype=np.int32)
    d, off = 0, 0
    for s in range(1, num_samples + 1):
        need = seq_length + 1
        while True:
            avail = sizes[doc_idx[d]] - off
            if avail >= need:
                off += need - 1
                break
            need -= avail
            d += 1
            off = 0
        out[s] = (d, off)
    return out


def _build_shuffle_idx(num_samples, total_size, np_rng):
    dtype = np.uint32 if total_size < np.iinfo(np.uint32).max - 1 else np.int64
    first = np.arange(0, num_samples, dtype=dtype)
    np_rng.shuffle(first)
    if num_samples == total_size:
        return first
    last = np.arange(num_samples, total_size, dtype=dtype)
    np_rng.shuffle(last)
    return np.concatenate((first, last))


def _save_atomic(path, arr):
    tmp = path + ".tmp.%d.npy" % os.getpid()
    np.save(tmp, arr, allow_pickle=False)
    os.replace(tmp, path)


def construct_samples_and_shuffle_data(name, data_prefix, documents, sizes, num_samples,
                                       seq_length, seed, build_data_file):
    tokens_per_epoch = int(np.sum(sizes[documents]))
    num_epochs = _num_epochs(tokens_per_epoch, seq_length, num_samples)
    np_rng = np.random.RandomState(seed=seed)
    base = "{}_{}_indexmap_{}ns_{}sl".format(data_prefix, name, num_samples, seq_length)
    doc_f, sample_f, shuffle_f = base + "_doc_idx.npy", base + "_sample_idx.npy", base + "_shuffle_idx.npy"
    if build_data_file:
        if not all(os.path.isfile(f) for f in (doc_f, sample_f, shuffle_f)):
            if num_epochs == 1:
                separate_last = False
            else:
                from_prev = ((num_epochs - 1) * tokens_per_epoch - 1) // seq_length
                last_epoch_samples = num_samples - from_prev
                per_epoch = (tokens_per_epoch - 1) // seq_length
                assert 0 <= last_epoch_samples < per_epoch + 1
                separate_last = last_epoch_samples < int(0.80 * per_epoch)
            t0 = time.time()
            doc_idx = _build_doc_idx(documents, num_epochs, np_rng, separate_last)
            _save_atomic(doc_f, doc_idx)
            sizes32 = sizes.astype(np.int32)
            try:
                from ..._C import _native
                sample_idx = _native.build_sample_idx(sizes32, doc_idx, seq_length, num_epochs,
                                                      tokens_per_epoch)
            except ImportError:
                logger.warning("native index builder not built; using the Python builder")
                sample_idx = build_sample_idx_py(sizes32, doc_idx, seq_length, num_epochs,
                                                 tokens_per_epoch)
            _save_atomic(sample_f, sample_idx)
            n_ = from_prev if separate_last else sample_idx.shape[0] - 1
            shuffle_idx = _build_shuffle_idx(n_, sample_idx.shape[0] - 1, np_rng)
            _save_atomic(shuffle_f, shuffle_idx)
            logger.info("built index maps for {} in {:.2f}s".format(name, time.time() - t0))
    else:
        while not all(os.path.isfile(f) for f in (doc_f, sample_f, shuffle_f)):
            time.sleep(1)
    _barrier()
    return (np.load(doc_f, mmap_mode="r"), np.load(sample_f, mmap_mode="r"),
            np.load(shuffle_f, mmap_mode="r"))


def _barrier():
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


class GPTDataset(torch.utils.data.Dataset):
    def __init__(self, input_dir, split, max_seq_len, num_samples, mode, seed=1234, eos_id=50256,
                 **kwargs):
        files = get_train_data_file(input_dir) if os.path.isdir(input_dir) else [input_dir]
        assert len(files) == 1, "GPT supports one dataset prefix"
        prefix = files[0]
        for suffix in ("_ids.npy", "_idx.npz"):
            if not os.path.isfile(prefix + suffix):
                raise ValueError("File not found: %s" % (prefix + suffix))
        self.sample_ids = np.load(prefix + "_ids.npy", mmap_mode="r")
        self.sample_lens = np.load(prefix + "_idx.npz")["lens"].astype(np.int32)
        splits = get_train_valid_test_split_(split, len(self.sample_lens))
        self.max_seq_len = max_seq_len
        self.mode = mode
        self.name = "gpt_" + mode
        self.eos_id = eos_id
        documents = np.arange(splits[MODE_TO_INDEX[mode]], splits[MODE_TO_INDEX[mode] + 1])
        self.doc_idx, self.sample_idx, self.shuffle_idx = construct_samples_and_shuffle_data(
            self.name, prefix, documents, self.sample_lens, num_samples, max_seq_len, seed,
            env.get_local_rank() == 0)
        self.start_pos = np.concatenate([[0], np.cumsum(self.sample_lens, dtype=np.int64)])

    def _construct_sample(self, tokens):
        tokens = np.asarray(tokens, dtype=np.int64)
        labels = tokens[1:]
        tokens = tokens[:-1]
        loss_mask = np.ones(len(tokens), dtype=np.float32)
        loss_mask[tokens == self.eos_id] = 0.0
        position_ids = np.arange(len(tokens), dtype=np.int64)
        if self.mode == "Test":
            return [tokens, position_ids]
        return [tokens, position_ids, labels, loss_mask]

    def _tokens(self, df, dl, of, ol):
        if df == dl:
            s = self.start_pos[self.doc_idx[df]]
            return self.sample_ids[s + of:s + ol + 1]
        parts = [self.sample_ids[self.start_pos[self.doc_idx[df]] + of:
                                 self.start_pos[self.doc_idx[df] + 1]]]
        for i in range(df + 1, dl):
            parts.append(self.sample_ids[self.start_pos[self.doc_idx[i]]:
                                         self.start_pos[self.doc_idx[i] + 1]])
        s = self.start_pos[self.doc_idx[dl]]
        parts.append(self.sample_ids[s:s + ol + 1])
        return np.concatenate(parts)

    def __getitem__(self, index):
        idx = int(self.shuffle_idx[index])
        df, of = self.sample_idx[idx]
        dl, ol = self.sample_idx[idx + 1]
        return self._construct_sample(self._tokens(int(df), int(dl), int(of), int(ol)))

    def __len__(self):
        return self.sample_idx.shape[0] - 1


class SyntheticGPTDataset(torch.utils.data.Dataset):
    """Random-token samples of the GPTDataset format (no files, no network).

    Token ``i`` of sample ``n`` is drawn from ``RandomState(seed + n)`` so the
    stream is identical for every parallel layout.
    """

    def __init__(self, max_seq_len, num_samples=10 ** 9, vocab_size=50304, seed=1234,
                 mode="Train", eos_id=50256, **kwargs):
        self.max_seq_len = max_seq_len
        self.num_samples = int(num_samples)
        self.vocab_size = vocab_size
        self.seed = seed
        self.mode = mode
        self.eos_id = eos_id

    def __len__(self):
        return self.num_samples

    def __getitem__(self, index):
        rs = np.random.RandomState((self.seed + int(index)) % (2 ** 32))
        toks = rs.randint(0, self.vocab_size, size=self.max_seq_len + 1).astype(np.int64)
        tokens, labels = toks[:-1], toks[1:]
        loss_mask = np.ones(self.max_seq_len, dtype=np.float32)
        loss_mask[tokens == self.eos_id] = 0.0
        pos = np.arange(self.max_seq_len, dtype=np.int64)
        if self.mode == "Test":
            return [tokens, pos]
        return [tokens, pos, labels, loss_mask]


def wikitext_detokenize(string):
    string = string.replace("s '", "s'")
    string = re.sub(r"/' [0-9]/", r"/'[0-9]/", string)
    for a, b in ((" @-@ ", "-"), (" @,@ ", ","), (" @.@ ", "."), (" : ", ": "), (" ; ", "; "),
                 (" . ", ". "), (" ! ", "! "), (" ? ", "? "), (" , ", ", ")):
        string = string.replace(a, b)
    string = re.sub(r"\(\s*([^\)]*?)\s*\)", r"(\1)", string)
    string = re.sub(r"\[\s*([^\]]*?)\s*\]", r"[\1]", string)
    string = re.sub(r"{\s*([^}]*?)\s*}", r"{\1}", string)
    string = re.sub(r"\"\s*([^\"]*?)\s*\"", r'"\1"', string)
    string = re.sub(r"'\s*([^']*?)\s*'", r"'\1'", string)
    for a, b in (("= = = =", "===="), ("= = =", "==="), ("= =", "=="),
                 (" " + chr(176) + " ", chr(176)), (" \n", "\n"), ("\n ", "\n"), (" N ", " 1 "),
                 (" 's", "'s")):
        string = string.replace(a, b)
    return string


def _tokenizer(kwargs):
    from ..tokenizers import GPTTokenizer
    return kwargs.get("tokenizer") or GPTTokenizer.from_pretrained(kwargs.get("vocab_dir", "gpt2"))


class LM_Eval_Dataset(torch.utils.data.Dataset):
    """WikiText PPL windows (reference ``gpt_dataset.py:462-559``)."""

    def __init__(self, input_dir, max_seq_len, overlapping_eval=None, **kwargs):
        tok = _tokenizer(kwargs)
        with open(input_dir, "rb") as f:
            data = f.read().decode("utf-8")
        self.num_original_tokens = len(data.strip().split(" "))
        data = wikitext_detokenize(data)
        self.tokens = tok.encode(data)
        self.num_tokenized_tokens = len(self.tokens)
        self.seq_len = max_seq_len
        self.pad_idx = tok.eos_token_id
        self.overlapping_eval = max(1, overlapping_eval or self.seq_len)
        self.total_targets = len(self.tokens) - 1
        targets = max(self.total_targets - self.overlapping_eval, 0)
        self.total_sequences = max(math.ceil(targets / self.overlapping_eval) + 1, 1)

    def __len__(self):
        return self.total_sequences

    def __getitem__(self, idx):
        start = idx * self.overlapping_eval
        toks = list(self.tokens[start:start + self.seq_len + 1])
        if len(toks) < self.seq_len + 1:
            toks += [self.pad_idx] * (self.seq_len + 1 - len(toks))
        toks = np.asarray(toks, dtype=np.int64)
        tokens, labels = toks[:-1], toks[1:]
        loss_mask = np.ones(self.seq_len, dtype=np.float32)
        loss_mask[tokens == self.pad_idx] = 0.0
        if self.overlapping_eval != self.seq_len and idx != 0:
            loss_mask[:-self.overlapping_eval] = 0.0
        attention_mask = np.tri(self.seq_len, self.seq_len, dtype=np.float32)[None]
        pos = np.arange(self.seq_len, dtype=np.int64)
        return [tokens, loss_mask, attention_mask, pos, labels,
                np.array([self.num_original_tokens, self.num_tokenized_tokens])]


class Lambada_Eval_Dataset(torch.utils.data.Dataset):
    """LAMBADA last-word cloze (reference ``gpt_dataset.py:562-627``)."""

    def __init__(self, input_dir, max_seq_len, **kwargs):
        tok = _tokenizer(kwargs)
        self.tokens, self.labels = [], []
        with open(input_dir, "r") as f:
            for line in f:
                text = json.loads(line)["text"]
                last = text.split()[-1]
                start = text.rfind(last)
                self.tokens.append(tok.encode(text[:start].strip()))
                self.labels.append(tok.encode(" " + last))
        self.pad_idx = tok.eos_token_id
        self.seq_len = max_seq_len

    def __len__(self):
        return len(self.tokens)

    def __getitem__(self, idx):
        toks = list(self.tokens[idx][:self.seq_len]) + list(self.labels[idx])
        n = len(toks)
        if n < self.seq_len + 1:
            toks += [self.pad_idx] * (self.seq_len + 1 - n)
        loss_mask = np.zeros(self.seq_len, dtype=np.float32)
        loss_mask[n - len(self.labels[idx]) - 1:n - 1] = 1.0
        toks = np.asarray(toks, dtype=np.int64)
        tokens, labels = toks[:-1], toks[1:]
        attention_mask = np.tri(self.seq_len, self.seq_len, dtype=np.float32)[None]
        pos = np.arange(self.seq_len, dtype=np.int64)
        return [tokens, loss_mask, attention_mask, pos, labels, np.array([len(self.tokens)])]
