"""Text-to-image datasets for Imagen.

Parity: reference ``data/dataset/multimodal_dataset.py:36-180`` (D10): the
input is a list file naming TSV shards; each rank takes every
``world_size``-th shard (padded so shards divide evenly); each TSV line holds
``<id>\\t<text_emb.npy>\\t<attn_mask.npy>\\t<base64 image>``, the ``.npy`` paths
relative to the shard.  Images are box-downsampled while >= 2x the target,
bicubic-resized so the short side equals ``input_resolusion`` and centre
cropped.  Line offsets are indexed once so ``__getitem__`` seeks directly.

The reference returns 0-255 floats that its ``cast_uint8_images_to_float``
never rescales; images are returned in [0, 1] here, the range the diffusion
normalisation expects.  ``.npy`` files are read with ``allow_pickle=False``.
``SyntheticImagenDataset`` provides random images / embeddings of the same
shapes for benchmarks and tests.
"""
import base64
import io
import os
import random

import numpy as np
from PIL import Image

from ...utils import env


def get_files(data_path, world_size, rank, shuffle=False, seed=0):
    with open(data_path) as f:
        files = [ln.strip() for ln in f if ln.strip()]
    base = os.path.dirname(os.path.abspath(data_path))
    files = [p if os.path.isabs(p) else os.path.join(base, p) for p in files]
    rng = random.Random(seed)
    if shuffle:
        rng.shuffle(files)
    if len(files) % world_size:
        extra = world_size - len(files) % world_size
        files = files + [files[i % len(files)] for i in range(extra)]
    return files[rank::world_size]


def augment_for_imagen(img, resolution):
    while min(*img.size) >= 2 * resolution:
        img = img.resize(tuple(x // 2 for x in img.size), resample=Image.BOX)
    scale = resolution / min(*img.size)
    img = img.resize(tuple(round(x * scale) for x in img.size), resample=Image.BICUBIC)
    arr = np.asarray(img.convert("RGB"))
    cy, cx = (arr.shape[0] - resolution) // 2, (arr.shape[1] - resolution) // 2
    arr = arr[cy:cy + resolution, cx:cx + resolution]
    return np.ascontiguousarray(arr.transpose(2, 0, 1)).astype(np.float32) / 255.0


class ImagenDataset:
    def __init__(self, input_path, input_format="embed_base64_cc12m", shuffle=False,
                 input_resolusion=64, second_size=256, max_seq_len=128,
                 filter_image_resolution=128, tokenizer=None, split="train", seed=1024, **kwargs):
        self.files = get_files(input_path, env.get_data_world_size(), env.get_data_world_rank(),
                               shuffle, seed)
        self.input_resolusion = input_resolusion
        self.max_seq_len = max_seq_len
        self.index = []
        for fi, path in enumerate(self.files):
            off = 0
            with open(path, "rb") as f:
                for line in f:
                    self.index.append((fi, off, len(line)))
                    off += len(line)
        if split == "train":
            random.Random(seed).shuffle(self.index)

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        fi, off, n = self.index[i]
        path = self.files[fi]
        with open(path, "rb") as f:
            f.seek(off)
            line = f.read(n).decode("utf-8")
        parts = line.rstrip("\n").split("\t")
        d = os.path.dirname(path)
        emb = np.load(os.path.join(d, parts[1]), mmap_mode="r", allow_pickle=False)
        mask = np.load(os.path.join(d, parts[2]), mmap_mode="r", allow_pickle=False)
        img = Image.open(io.BytesIO(base64.b64decode(parts[3])))
        emb = np.asarray(emb[:self.max_seq_len], dtype=np.float32)
        mask = np.asarray(mask[:self.max_seq_len]).astype(np.int64)
        return augment_for_imagen(img, self.input_resolusion), emb, mask


class SyntheticImagenDataset:
    """Random images in [0,1] + text embeddings with random valid lengths."""

    def __init__(self, num_samples=100000, input_resolusion=64, max_seq_len=128,
                 text_embed_dim=1024, seed=0, **kwargs):
        self.n, self.res, self.L, self.D, self.seed = num_samples, input_resolusion, max_seq_len, \
            text_embed_dim, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        rs = np.random.RandomState((self.seed * 7919 + i) & 0x7FFFFFFF)
        img = rs.rand(3, self.res, self.res).astype(np.float32)
        n = rs.randint(self.L // 4, self.L + 1)
        emb = np.zeros((self.L, self.D), np.float32)
        emb[:n] = rs.standard_normal((n, self.D)).astype(np.float32)
        mask = np.zeros(self.L, np.int64)
        mask[:n] = 1
        return img, emb, mask
