"""Image-classification datasets.

Parity: reference ``data/dataset/vision_dataset.py:25-357`` (D04):
``GeneralClsDataset`` (``root`` + ``"path label"`` list file, optional
multi-label one-hot), ``ImageFolder`` (class-per-subdirectory layout) and
``CIFAR`` (CIFAR-10 batches).  Added: ``SyntheticImageDataset`` for
benchmarks without data on disk (no network here).

CIFAR: the reference unpickles the python batches.  Here the binary batches
(``data_batch_N.bin`` / ``test_batch.bin``, 1 label byte + 3072 pixel bytes)
are read directly, and the python batches are read through a restricted
unpickler that only admits plain containers and numpy array reconstruction.
"""
import io
import os
import pickle

import numpy as np

from ...utils.log import logger
from ..transforms import create_preprocess_operators, transform

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


class _Retry:
    """Corrupt sample -> log and serve a random other one (reference behaviour)."""

    def _get(self, idx):
        raise NotImplementedError

    def __getitem__(self, idx):
        for _ in range(10):
            try:
                return self._get(idx)
            except Exception as ex:  # noqa: BLE001 - matches the reference's catch-all
                logger.error("Exception occured when parse sample {}: {}".format(idx, ex))
                idx = np.random.randint(len(self))
        raise RuntimeError("too many unreadable samples")


class GeneralClsDataset(_Retry):
    def __init__(self, image_root, cls_label_path, transform_ops=None, delimiter=" ",
                 multi_label=False, class_num=None):
        if multi_label:
            assert class_num is not None, "Must set class_num when multi_label=True"
        self.multi_label, self.classes_num = multi_label, class_num
        self._img_root, self._cls_path, self.delimiter = image_root, cls_label_path, delimiter
        self._ops = create_preprocess_operators(transform_ops) if transform_ops else None
        self.images, self.labels = [], []
        assert os.path.exists(cls_label_path), "%s does not exist" % cls_label_path
        assert os.path.exists(image_root), "%s does not exist" % image_root
        with open(cls_label_path) as f:
            for line in f:
                parts = line.strip().split(self.delimiter)
                if len(parts) < 2:
                    continue
                self.images.append(os.path.join(image_root, parts[0]))
                self.labels.append(parts[1] if multi_label else np.int32(parts[1]))
                assert os.path.exists(self.images[-1]), "%s does not exist" % self.images[-1]

    def _get(self, idx):
        with open(self.images[idx], "rb") as f:
            img = f.read()
        if self._ops:
            img = transform(img, self._ops)
        if self.multi_label:
            oh = np.zeros([self.classes_num], dtype=np.float32)
            for c in self.labels[idx].split(","):
                oh[int(c)] = 1.0
            return img, oh
        return img, np.int32(self.labels[idx])

    def __len__(self):
        return len(self.images)

    @property
    def class_num(self):
        return self.classes_num if self.multi_label else len(set(self.labels))


class ImageFolder(_Retry):
    def __init__(self, root, extensions=IMG_EXTENSIONS, transform_ops=None):
        self.root = root
        self.classes = sorted(e.name for e in os.scandir(root) if e.is_dir())
        if not self.classes:
            raise FileNotFoundError("Couldn't find any class folder in %s." % root)
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        exts = tuple(e.lower() for e in extensions)
        self.imgs = []
        for c in self.classes:
            found = False
            for r, _, fnames in sorted(os.walk(os.path.join(root, c), followlinks=True)):
                for fn in sorted(fnames):
                    if fn.lower().endswith(exts):
                        self.imgs.append((os.path.join(r, fn), self.class_to_idx[c]))
                        found = True
            if not found:
                raise FileNotFoundError("Found no valid file for the class %s" % c)
        self.targets = [t for _, t in self.imgs]
        self._ops = create_preprocess_operators(transform_ops) if transform_ops else None
        logger.info("find total %d classes and %d images." % (len(self.classes), len(self.imgs)))

    def _get(self, idx):
        path, target = self.imgs[idx]
        with open(path, "rb") as f:
            img = f.read()
        if self._ops:
            img = transform(img, self._ops)
        return img, np.int32(target)

    def __len__(self):
        return len(self.imgs)

    @property
    def class_num(self):
        return len(self.classes)


class _NumpyOnlyUnpickler(pickle.Unpickler):
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError("refusing to load %s.%s" % (module, name))


def _read_cifar_batch(path):
    if path.endswith(".bin"):
        raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 3073)
        return raw[:, 1:].reshape(-1, 3, 32, 32), raw[:, 0].astype(np.int64)
    with open(path, "rb") as f:
        d = _NumpyOnlyUnpickler(io.BytesIO(f.read()), encoding="bytes").load()
    return np.asarray(d[b"data"]).reshape(-1, 3, 32, 32), np.asarray(d[b"labels"])


class CIFAR:
    def __init__(self, root, mode="train", transform_ops=None):
        assert mode in ("train", "test")
        self.root, self.mode = root, mode
        self._ops = create_preprocess_operators(transform_ops) if transform_ops else None
        names = ["data_batch_%d" % i for i in range(1, 6)] if mode == "train" else ["test_batch"]
        imgs, labels = [], []
        for n in names:
            p = os.path.join(root, n)
            if not os.path.exists(p) and os.path.exists(p + ".bin"):
                p += ".bin"
            x, y = _read_cifar_batch(p)
            imgs.append(x.transpose(0, 2, 3, 1))
            labels.append(y)
        self.images = np.ascontiguousarray(np.concatenate(imgs))
        self.labels = np.concatenate(labels)

    def __getitem__(self, idx):
        img = self.images[idx]
        if self._ops:
            img = transform(img, self._ops)
        return img, np.int32(self.labels[idx])

    def __len__(self):
        return len(self.images)

    @property
    def class_num(self):
        return len(set(self.labels.tolist()))


class SyntheticImageDataset:
    """Deterministic random images/labels of a given shape (benchmarks, tests)."""

    def __init__(self, num_samples=1024, image_size=224, class_num=1000, channels=3, seed=0,
                 dtype="float32", **kwargs):
        self.n, self.size, self.classes, self.c = num_samples, image_size, class_num, channels
        self.seed, self.dtype = seed, dtype

    def __getitem__(self, idx):
        rs = np.random.RandomState((self.seed * 1000003 + idx) & 0x7FFFFFFF)
        img = rs.standard_normal((self.c, self.size, self.size)).astype(self.dtype)
        return img, np.int32(rs.randint(self.classes))

    def __len__(self):
        return self.n

    @property
    def class_num(self):
        return self.classes
