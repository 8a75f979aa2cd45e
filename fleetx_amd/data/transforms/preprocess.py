"""Image preprocessing operators (HWC uint8 numpy in, numpy out).

Parity: reference ``data/transforms/preprocess.py:37-380`` (D06): DecodeImage,
ResizeImage (resize_short / size), CenterCropImage, RandCropImage
(scale/aspect sampled crop + resize), RandFlipImage, NormalizeImage,
ToCHWImage, ColorJitter, RandomErasing.  The reference decodes and resizes
with OpenCV; OpenCV is not part of this image, so decoding and resizing go
through PIL (the reference's own ``backend: pil`` path) and flips/crops are
numpy slicing.  Arithmetic strings in configs (``scale: 1.0/255.0``) are
evaluated by a literal-arithmetic parser, never ``eval``.
"""
import ast
import io
import math
import operator
import random

import numpy as np
from PIL import Image, ImageEnhance

_OPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul,
        ast.Div: operator.truediv, ast.Pow: operator.pow, ast.USub: operator.neg,
        ast.UAdd: operator.pos}


def arith(v):
    """Evaluate a numeric literal expression such as ``'1.0/255.0'``."""
    if not isinstance(v, str):
        return v

    def ev(node):
        if isinstance(node, ast.Expression):
            return ev(node.body)
        if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)):
            return node.value
        if isinstance(node, ast.BinOp) and type(node.op) in _OPS:
            return _OPS[type(node.op)](ev(node.left), ev(node.right))
        if isinstance(node, ast.UnaryOp) and type(node.op) in _OPS:
            return _OPS[type(node.op)](ev(node.operand))
        raise ValueError("not a numeric expression: %r" % v)
    return ev(ast.parse(v, mode="eval"))


class OperatorParamError(ValueError):
    pass


_PIL_INTERP = {"nearest": Image.NEAREST, "bilinear": Image.BILINEAR, "bicubic": Image.BICUBIC,
               "box": Image.BOX, "lanczos": Image.LANCZOS, "hamming": Image.HAMMING,
               "area": Image.BOX}


class UnifiedResize:
    """``(src HWC array, (w, h)) -> resized array`` (PIL resampling)."""

    def __init__(self, interpolation=None, backend="pil"):
        if isinstance(interpolation, str):
            interpolation = _PIL_INTERP[interpolation.lower()]
        self.resample = Image.BILINEAR if interpolation is None else interpolation

    def __call__(self, src, size):
        return np.asarray(Image.fromarray(np.ascontiguousarray(src)).resize(tuple(size),
                                                                            self.resample))


class DecodeImage:
    def __init__(self, to_rgb=True, channel_first=False):
        self.to_rgb, self.channel_first = to_rgb, channel_first

    def __call__(self, img):
        assert isinstance(img, (bytes, bytearray)) and len(img) > 0, "invalid input to DecodeImage"
        im = Image.open(io.BytesIO(img)).convert("RGB")
        arr = np.asarray(im)
        if not self.to_rgb:  # reference decodes BGR and flips to RGB
            arr = arr[:, :, ::-1]
        if self.channel_first:
            arr = arr.transpose((2, 0, 1))
        return np.ascontiguousarray(arr)


class ResizeImage:
    def __init__(self, size=None, resize_short=None, interpolation=None, backend="pil"):
        if resize_short is not None and resize_short > 0:
            self.resize_short, self.w, self.h = resize_short, None, None
        elif size is not None:
            self.resize_short = None
            self.w = size if isinstance(size, int) else size[0]
            self.h = size if isinstance(size, int) else size[1]
        else:
            raise OperatorParamError("ResizeImage needs 'size' or 'resize_short'")
        self._resize = UnifiedResize(interpolation, backend)

    def __call__(self, img):
        ih, iw = img.shape[:2]
        if self.resize_short is not None:
            pct = float(self.resize_short) / min(iw, ih)
            w, h = int(round(iw * pct)), int(round(ih * pct))
        else:
            w, h = self.w, self.h
        return self._resize(img, (w, h))


class CenterCropImage:
    def __init__(self, size):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def __call__(self, img):
        w, h = self.size
        ih, iw = img.shape[:2]
        ws, hs = (iw - w) // 2, (ih - h) // 2
        return img[hs:hs + h, ws:ws + w, :]


class RandCropImage:
    """Inception-style crop: area in ``scale`` x image, aspect in ``ratio``."""

    def __init__(self, size, scale=None, ratio=None, interpolation=None, backend="pil"):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.scale = [0.08, 1.0] if scale is None else scale
        self.ratio = [3.0 / 4.0, 4.0 / 3.0] if ratio is None else ratio
        self._resize = UnifiedResize(interpolation, backend)

    def __call__(self, img):
        ar = math.sqrt(random.uniform(*self.ratio))
        fw, fh = ar, 1.0 / ar
        ih, iw = img.shape[:2]
        bound = min((float(iw) / ih) / (fw ** 2), (float(ih) / iw) / (fh ** 2))
        smax, smin = min(self.scale[1], bound), min(self.scale[0], bound)
        side = math.sqrt(iw * ih * random.uniform(smin, smax))
        w, h = int(side * fw), int(side * fh)
        x = random.randint(0, iw - w)
        y = random.randint(0, ih - h)
        return self._resize(img[y:y + h, x:x + w, :], self.size)


class RandFlipImage:
    """flip_code 1: horizontal, 0: vertical, -1: both (applied with p=0.5)."""

    def __init__(self, flip_code=1):
        assert flip_code in (-1, 0, 1)
        self.flip_code = flip_code

    def __call__(self, img):
        if random.randint(0, 1) != 1:
            return img
        if self.flip_code == 1:
            return img[:, ::-1]
        if self.flip_code == 0:
            return img[::-1]
        return img[::-1, ::-1]


class NormalizeImage:
    def __init__(self, scale=None, mean=None, std=None, order="chw", output_fp16=False,
                 channel_num=3):
        assert channel_num in (3, 4)
        self.channel_num = channel_num
        self.dtype = "float16" if output_fp16 else "float32"
        self.scale = np.float32(arith(scale) if scale is not None else 1.0 / 255.0)
        self.order = order
        mean = mean if mean is not None else [0.485, 0.456, 0.406]
        std = std if std is not None else [0.229, 0.224, 0.225]
        shape = (3, 1, 1) if order == "chw" else (1, 1, 3)
        self.mean = np.array(mean, dtype="float32").reshape(shape)
        self.std = np.array(std, dtype="float32").reshape(shape)

    def __call__(self, img):
        img = np.asarray(img)
        img = (img.astype("float32") * self.scale - self.mean) / self.std
        if self.channel_num == 4:
            ax = 0 if self.order == "chw" else 2
            shp = list(img.shape)
            shp[ax] = 1
            img = np.concatenate([img, np.zeros(shp, dtype=img.dtype)], axis=ax)
        return img.astype(self.dtype)


class ToCHWImage:
    def __call__(self, img):
        return np.ascontiguousarray(np.asarray(img).transpose((2, 0, 1)))


class ColorJitter:
    """Brightness / contrast / saturation / hue jitter in random order."""

    def __init__(self, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.0):
        self.b, self.c, self.s, self.h = brightness, contrast, saturation, hue

    @staticmethod
    def _factor(v):
        return random.uniform(max(0.0, 1 - v), 1 + v)

    def __call__(self, img):
        im = img if isinstance(img, Image.Image) else Image.fromarray(np.ascontiguousarray(img))
        fns = []
        if self.b:
            fns.append(lambda x: ImageEnhance.Brightness(x).enhance(self._factor(self.b)))
        if self.c:
            fns.append(lambda x: ImageEnhance.Contrast(x).enhance(self._factor(self.c)))
        if self.s:
            fns.append(lambda x: ImageEnhance.Color(x).enhance(self._factor(self.s)))
        if self.h:
            def hue(x):
                shift = random.uniform(-self.h, self.h)
                hsv = np.array(x.convert("HSV"))
                hsv[..., 0] = (hsv[..., 0].astype(np.int32) + int(shift * 255)) % 256
                return Image.fromarray(hsv, "HSV").convert("RGB")
            fns.append(hue)
        random.shuffle(fns)
        for f in fns:
            im = f(im)
        return np.asarray(im)


class Pixels:
    def __init__(self, mode="const", mean=(0.0, 0.0, 0.0)):
        self.mode, self.mean = mode, list(mean)

    def __call__(self, h=224, w=224, c=3):
        if self.mode == "rand":
            return np.random.normal(size=(1, 1, 3))
        if self.mode == "pixel":
            return np.random.normal(size=(h, w, c))
        if self.mode == "const":
            return self.mean
        raise ValueError("RandomErasing mode must be const / rand / pixel")


class RandomErasing:
    def __init__(self, EPSILON=0.5, sl=0.02, sh=0.4, r1=0.3, mean=(0.0, 0.0, 0.0), attempt=100,
                 use_log_aspect=False, mode="const"):
        self.EPSILON, self.sl, self.sh = arith(EPSILON), arith(sl), arith(sh)
        r1 = arith(r1)
        self.r1 = (math.log(r1), math.log(1 / r1)) if use_log_aspect else (r1, 1 / r1)
        self.use_log_aspect, self.attempt = use_log_aspect, attempt
        self.get_pixels = Pixels(mode, mean)

    def __call__(self, img):
        if random.random() > self.EPSILON:
            return img
        img = np.array(img)
        for _ in range(self.attempt):
            area = img.shape[0] * img.shape[1]
            target = random.uniform(self.sl, self.sh) * area
            ar = random.uniform(*self.r1)
            if self.use_log_aspect:
                ar = math.exp(ar)
            h = int(round(math.sqrt(target * ar)))
            w = int(round(math.sqrt(target / ar)))
            if w < img.shape[1] and h < img.shape[0]:
                px = self.get_pixels(h, w, img.shape[2])
                x1 = random.randint(0, img.shape[0] - h)
                y1 = random.randint(0, img.shape[1] - w)
                if img.shape[2] == 3:
                    img[x1:x1 + h, y1:y1 + w, :] = px
                else:
                    img[x1:x1 + h, y1:y1 + w, 0] = px[0]
                return img
        return img
