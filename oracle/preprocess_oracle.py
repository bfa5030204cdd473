"""CPU ORACLE for the image preprocessing row — test infrastructure only.

Restates, in NumPy, the two eval preprocessing pipelines the reference runs on the host:

* CLIP eval (open_clip/src/open_clip/transform.py:371-389, image_transform with resize_mode
  'shortest', is_train=False): torchvision Resize(336, BICUBIC) on a PIL image -> Pillow's
  two-pass resampler (third-party: Pillow, src/libImaging/Resample.c, unpinned by the reference;
  12.2.0 in this container) -> CenterCrop(336) -> ToTensor -> Normalize(OpenAI mean/std,
  constants.py:1-2).  Pillow resamples uint8 in fixed point (22 fractional bits), horizontal pass
  first, so the restatement below is integer-exact and the device kernel is checked bit-exactly.
* PACL eval (Patch-Aligned-Contrastive-Learning/data/utils.py:30-37): ToTensor -> Resize((336,
  336)) on the float tensor -> torch.nn.functional.interpolate(bilinear, antialias=True)
  (torchvision >= 0.17 default; third-party torch ATen UpSampleKernel.cpp separable AA kernel,
  width pass first) -> Normalize(ImageNet mean/std).  Float arithmetic: checked to a tolerance.

Pinned by tests/test_oracle_preprocess.py against Pillow and torch in this container and by the
committed fixtures tests/golden/preprocess.npz (made by tests/golden/make_golden_preprocess.py).
Never imported by the product.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
PRECISION_BITS = 32 - 8 - 2
OPENAI_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_STD = (0.26862954, 0.26130258, 0.27577711)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ------------------------------------------------------------------ Pillow bicubic (Resample.c)
def _bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def pil_coeffs(in_size: int, out_size: int):
    """precompute_coeffs + normalize_coeffs_8bpc: per output index (xmin, xsize, int32 taps)."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)          # C cast truncates toward zero
        xmin = max(xmin, 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)                                   # sequential double sum, as the C loop
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(ss: np.ndarray) -> np.ndarray:
    return np.clip(ss >> PRECISION_BITS, 0, 255).astype(np.uint8)


def pil_resize_bicubic(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """Image.resize((out_w, out_h), BICUBIC) for an RGB uint8 [H,W,3] array."""
    H, W, _ = img.shape
    x = img.astype(np.int64)
    if out_w != W:
        b, k = pil_coeffs(W, out_w)
        out = np.empty((H, out_w, 3), np.uint8)
        for xx in range(out_w):
            xmin, n = b[xx]
            ss = (1 << (PRECISION_BITS - 1)) + np.einsum("hkc,k->hc", x[:, xmin:xmin + n, :], k[xx, :n])
            out[:, xx, :] = _clip8(ss)
        x = out.astype(np.int64)
    if out_h != H:
        b, k = pil_coeffs(H, out_h)
        out = np.empty((out_h, x.shape[1], 3), np.uint8)
        for yy in range(out_h):
            ymin, n = b[yy]
            ss = (1 << (PRECISION_BITS - 1)) + np.einsum("kwc,k->wc", x[ymin:ymin + n, :, :], k[yy, :n])
            out[yy] = _clip8(ss)
        x = out.astype(np.int64)
    return x.astype(np.uint8)


def shortest_edge_size(h: int, w: int, size: int):
    """torchvision _compute_resized_output_size for Resize(int): (new_h, new_w)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    new_w, new_h = (new_short, new_long) if w <= h else (new_long, new_short)
    return new_h, new_w


def center_crop_offsets(h: int, w: int, size: int):
    """torchvision center_crop: int(round(...)) — Python's round-half-even."""
    return int(round((h - size) / 2.0)), int(round((w - size) / 2.0))


def to_tensor_normalize(u8_hwc: np.ndarray, mean, std) -> np.ndarray:
    x = u8_hwc.transpose(2, 0, 1).astype(F32) / F32(255)
    m = np.asarray(mean, F32)[:, None, None]
    s = np.asarray(std, F32)[:, None, None]
    return ((x - m) / s).astype(F32)


def clip_eval_preprocess(img: np.ndarray, size: int = 336) -> np.ndarray:
    """transform.py:371-389 on an RGB uint8 [H,W,3] image -> f32 [3,size,size]."""
    H, W, _ = img.shape
    nh, nw = shortest_edge_size(H, W, size)
    r = img if (nh, nw) == (H, W) else pil_resize_bicubic(img, nw, nh)
    top, left = center_crop_offsets(nh, nw, size)
    return to_tensor_normalize(r[top:top + size, left:left + size], OPENAI_MEAN, OPENAI_STD)


def clip_train_preprocess(img: np.ndarray, box, size: int = 336) -> np.ndarray:
    """open_clip's training preprocess (transform.py:334-355) for a given RandomResizedCrop box
    (top, left, height, width): torchvision F.resized_crop on a PIL image = Image.crop then
    Image.resize((size, size), BICUBIC), then ToTensor -> Normalize(OpenAI)."""
    top, left, h, w = (int(v) for v in box)
    crop = np.ascontiguousarray(img[top:top + h, left:left + w])
    r = crop if (h, w) == (size, size) else pil_resize_bicubic(crop, size, size)
    return to_tensor_normalize(r, OPENAI_MEAN, OPENAI_STD)


# ------------------------------------------------------------------ torch antialiased bilinear
def aa_bilinear_weights(in_size: int, out_size: int):
    """ATen _compute_weights_aa (bilinear, align_corners=False) in float32: (xmin, xsize, w)."""
    scale = F32(in_size) / F32(out_size)
    support = scale if scale >= 1.0 else F32(1.0)
    invscale = F32(1.0 / float(scale)) if scale >= 1.0 else F32(1.0)
    ksize = int(math.ceil(float(support))) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    wts = np.zeros((out_size, ksize), F32)
    for i in range(out_size):
        center = F32(float(scale) * (i + 0.5))                       # double product -> float
        xmin = max(int(float(F32(center - support)) + 0.5), 0)        # float diff, + 0.5 in double
        xsize = min(int(float(F32(center + support)) + 0.5), in_size) - xmin
        w = []
        for j in range(xsize):
            t = abs(F32((float(F32(F32(j + xmin) - center)) + 0.5) * float(invscale)))
            w.append(F32(1.0) - t if t < 1.0 else F32(0.0))
        tot = F32(0.0)
        for v in w:
            tot = F32(tot + v)
        if tot != 0.0:
            w = [F32(v / tot) for v in w]
        wts[i, :xsize] = w
        bounds[i] = (xmin, xsize)
    return bounds, wts


def aa_bilinear_resize(x_chw: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """interpolate(mode='bilinear', antialias=True) on f32 [C,H,W]: width pass, then height."""
    C, H, W = x_chw.shape
    x = x_chw.astype(F32)
    if out_w != W:
        b, w = aa_bilinear_weights(W, out_w)
        out = np.zeros((C, H, out_w), F32)
        for xx in range(out_w):
            xmin, n = b[xx]
            acc = x[:, :, xmin] * w[xx, 0]
            for j in range(1, n):
                acc = (acc + x[:, :, xmin + j] * w[xx, j]).astype(F32)
            out[:, :, xx] = acc
        x = out
    if out_h != H:
        b, w = aa_bilinear_weights(H, out_h)
        out = np.zeros((C, out_h, x.shape[2]), F32)
        for yy in range(out_h):
            ymin, n = b[yy]
            acc = x[:, ymin, :] * w[yy, 0]
            for j in range(1, n):
                acc = (acc + x[:, ymin + j, :] * w[yy, j]).astype(F32)
            out[:, yy, :] = acc
        x = out
    return x


def pacl_eval_preprocess(img: np.ndarray, size: int = 336) -> np.ndarray:
    """data/utils.py:33-37: ToTensor -> Resize((size,size)) (bilinear AA) -> Normalize(ImageNet)."""
    x = img.transpose(2, 0, 1).astype(F32) / F32(255)
    r = aa_bilinear_resize(x, size, size)
    m = np.asarray(IMAGENET_MEAN, F32)[:, None, None]
    s = np.asarray(IMAGENET_STD, F32)[:, None, None]
    return ((r - m) / s).astype(F32)
