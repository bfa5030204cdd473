"""Eval image preprocessing on the device — mirrors the reference's host transforms.

  image_transform(336, is_train=False)   open_clip/src/open_clip/transform.py:274-389 (eval path,
                                         resize_mode 'shortest', bicubic): Resize -> CenterCrop ->
                                         ToTensor -> Normalize(OpenAI)
  image_transform(336, is_train=True)    transform.py:334-355: RandomResizedCrop(scale=(0.9, 1.0),
                                         BICUBIC) -> ToTensor -> Normalize(OpenAI); box from the
                                         host torch RNG, resample on the device
  prepare_data(...).preprocess_image     Patch-Aligned-Contrastive-Learning/data/utils.py:30-52:
                                         ToTensor -> Resize((S,S)) -> Normalize(ImageNet)

Both run in libclipembed (ce_preprocess_images); the CLIP path reproduces Pillow's fixed-point
bicubic resampler bit for bit.  Inputs: PIL images, uint8 HWC numpy arrays or uint8 HWC tensors
(RGB), one at a time (-> [3,S,S], as the reference's transform) or a list (-> [B,3,S,S] in one
launch).  JPEG/PNG decoding stays on the host.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from .model import _ptr, _stream, kernel_engine


def _as_hwc_u8(img) -> np.ndarray:
    if isinstance(img, torch.Tensor):
        a = img.detach().cpu().numpy()
    elif isinstance(img, np.ndarray):
        a = img
    else:  # PIL.Image (convert('RGB') as _convert_to_rgb, transform.py:238-239)
        a = np.asarray(img.convert("RGB"))
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"expected an RGB uint8 HWC image, got dtype {a.dtype} shape {a.shape}")
    return np.ascontiguousarray(a)


class DeviceImageProcessor:
    """Callable like the reference's torchvision Compose; output on the device."""

    def __init__(self, mode: int, image_size: int = 336, device=None, out_dtype=torch.float32, engine=None):
        if image_size != 336 and engine is None:
            raise ValueError("the default kernel handle is configured for 336-pixel inputs; pass an engine")
        self.mode = mode
        self.image_size = image_size
        self.device = torch.device(device) if device is not None else None   # None: current device at call
        self.out_dtype = out_dtype
        self.engine = engine

    def __call__(self, image):
        batch = isinstance(image, (list, tuple))
        imgs = [_as_hwc_u8(x) for x in (image if batch else [image])]
        out = self.batch(imgs)
        return out if batch else out[0]

    @torch.no_grad()
    def batch(self, imgs: Sequence[np.ndarray]) -> torch.Tensor:
        return self._run(imgs, None)

    def _run(self, imgs: Sequence[np.ndarray], boxes: Optional[np.ndarray]) -> torch.Tensor:
        dev = self.device if self.device is not None else torch.device("cuda", torch.cuda.current_device())
        e = self.engine if self.engine is not None else kernel_engine(dev)
        sizes = [x.nbytes for x in imgs]
        offsets = np.zeros(len(imgs), np.int64)
        offsets[1:] = np.cumsum(sizes)[:-1]
        host = torch.empty(int(sum(sizes)), dtype=torch.uint8, pin_memory=True)
        hv = host.numpy()
        for x, o in zip(imgs, offsets):
            hv[o:o + x.nbytes] = x.reshape(-1)
        dev = host.to(e.device, non_blocking=True)
        heights = np.array([x.shape[0] for x in imgs], np.int32)
        widths = np.array([x.shape[1] for x in imgs], np.int32)
        S = self.image_size
        out = torch.empty(len(imgs), 3, S, S, device=e.device, dtype=self.out_dtype)
        dt = _lib.CE_BF16 if self.out_dtype == torch.bfloat16 else _lib.CE_F32
        if boxes is None:
            _lib.call("ce_preprocess_images", e.h, _stream(e.device), _ptr(dev), offsets.ctypes.data,
                      heights.ctypes.data, widths.ctypes.data, len(imgs), self.mode, dt, _ptr(out))
        else:
            boxes = np.ascontiguousarray(boxes, np.int32)
            _lib.call("ce_preprocess_images_boxes", e.h, _stream(e.device), _ptr(dev), offsets.ctypes.data,
                      heights.ctypes.data, widths.ctypes.data, boxes.ctypes.data, len(imgs), dt, _ptr(out))
        dev.record_stream(torch.cuda.current_stream(e.device))
        return out


def random_resized_crop_params(height: int, width: int, scale=(0.9, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0),
                               generator: Optional[torch.Generator] = None):
    """torchvision RandomResizedCrop.get_params (third-party, the transform open_clip's training
    preprocess builds, transform.py:334-340; torchvision is not imported here): the same torch RNG
    draws in the same order — per attempt two uniform_ draws, then two randint draws on success —
    so a seeded run picks the reference's boxes.  Returns (top, left, height, width)."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=generator).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1], generator=generator)).item()
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = torch.randint(0, height - h + 1, size=(1,), generator=generator).item()
            j = torch.randint(0, width - w + 1, size=(1,), generator=generator).item()
            return i, j, h, w
    in_ratio = float(width) / float(height)           # fallback: central crop
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


class DeviceTrainProcessor(DeviceImageProcessor):
    """open_clip's training preprocess (transform.py:334-355 with the default AugmentationCfg:
    RandomResizedCrop(S, scale=(0.9, 1.0), BICUBIC) -> RGB -> ToTensor -> Normalize(OpenAI)): the crop
    box is drawn on the host from the torch RNG (random_resized_crop_params, one image at a time in
    list order, as the reference's per-image calls do), the bicubic resample of the box runs on the
    device (ce_preprocess_images_boxes, Pillow-exact).  eval_clip.py:21-24 feeds this object to
    prepare_data_clip, so it is what the What'sUp / MMVP drivers preprocess with."""

    def __init__(self, image_size: int = 336, scale=(0.9, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0), device=None,
                 out_dtype=torch.float32, engine=None, generator: Optional[torch.Generator] = None):
        super().__init__(_lib.CE_PRE_CLIP_BICUBIC, image_size, device, out_dtype, engine)
        self.scale, self.ratio, self.generator = tuple(scale), tuple(ratio), generator

    @torch.no_grad()
    def batch(self, imgs: Sequence[np.ndarray]) -> torch.Tensor:
        boxes = np.array([random_resized_crop_params(x.shape[0], x.shape[1], self.scale, self.ratio, self.generator)
                          for x in imgs], np.int32).reshape(-1, 4)
        self.last_boxes = boxes          # (top, left, height, width) per image of the last call
        return self._run(imgs, boxes)


def image_transform(image_size=336, is_train: bool = False, mean: Optional[Sequence[float]] = None,
                    std: Optional[Sequence[float]] = None, resize_mode: Optional[str] = None,
                    interpolation: Optional[str] = None, fill_color: int = 0, aug_cfg=None, device=None,
                    engine=None):
    """open_clip image_transform (transform.py:274-389), eval path on the device."""
    from .weights import OPENAI_MEAN, OPENAI_STD
    if isinstance(image_size, (tuple, list)):
        if image_size[0] != image_size[1]:
            raise NotImplementedError("non-square image_size (ResizeKeepRatio) is not on the device path")
        image_size = image_size[0]
    if is_train:
        # open_clip's default AugmentationCfg (transform.py:62-72,334-355); jitter / grayscale / timm
        # augmentations are not on the device path
        # RandomResizedCrop gets `scale` only (transform.py:334-340): a `ratio` in aug_cfg is one of
        # the "Unused augmentation cfg items" the reference warns about (:356-357), so the default
        # (3/4, 4/3) stays and the seeded boxes match the reference's
        scale, ratio = (0.9, 1.0), (3.0 / 4.0, 4.0 / 3.0)
        if aug_cfg is not None:
            cfg = aug_cfg if isinstance(aug_cfg, dict) else vars(aug_cfg)
            extra = {k for k, v in cfg.items() if v and k not in ("scale", "ratio", "use_timm")}
            if extra or cfg.get("use_timm"):
                raise NotImplementedError(f"training augmentations {sorted(extra | ({'use_timm'} if cfg.get('use_timm') else set()))} "
                                          "are not on the device path")
            scale = tuple(cfg.get("scale") or scale)
            if cfg.get("ratio"):
                import warnings
                warnings.warn("Unused augmentation cfg items, specify `use_timm` to use (['ratio']).")
        if (mean is not None and tuple(mean) != tuple(OPENAI_MEAN)) or (std is not None and tuple(std) != tuple(OPENAI_STD)):
            raise NotImplementedError("the device path normalises with the OpenAI mean/std (constants.py:1-2)")
        return DeviceTrainProcessor(image_size, scale, ratio, device, engine=engine)
    if (resize_mode or "shortest") != "shortest" or (interpolation or "bicubic") != "bicubic":
        raise NotImplementedError("only resize_mode='shortest' with bicubic interpolation is on the device path")
    if (mean is not None and tuple(mean) != tuple(OPENAI_MEAN)) or (std is not None and tuple(std) != tuple(OPENAI_STD)):
        raise NotImplementedError("the device path normalises with the OpenAI mean/std (constants.py:1-2)")
    return DeviceImageProcessor(_lib.CE_PRE_CLIP_BICUBIC, image_size, device, engine=engine)


class _TextHalf:
    """preprocess_text of the reference's prepare_data classes (data/utils.py:54-55, 69-70): the
    ViT-L-14-336 tokenizer, here the C++ CLIP BPE (clipembed.tokenizer).  Created on first use, so
    the image half works where no BPE vocabulary file is available."""

    _tokenizer = None

    @property
    def tokenizer(self):
        if self._tokenizer is None:
            from .tokenizer import get_tokenizer
            self._tokenizer = get_tokenizer("ViT-L-14-336")
        return self._tokenizer

    def preprocess_text(self, caption):
        return self.tokenizer(caption)


class prepare_data(_TextHalf):
    """PACL prepare_data (data/utils.py:30-55): preprocess_image on the device, preprocess_text
    through the C++ tokenizer."""

    def __init__(self, base_model: str = "ViT-L-14-336", device=None, engine=None):
        if base_model != "ViT-L-14-336":
            raise NotImplementedError("only the ViT-L-14-336 (336 px) pipeline is on the device path")
        self.val_transform = DeviceImageProcessor(_lib.CE_PRE_PACL_BILINEAR_AA, 336, device, engine=engine)

    def preprocess_image(self, image):
        return self.val_transform(image)     # a list -> one batched launch, as torch.stack of the reference


class prepare_data_clip(_TextHalf):
    """prepare_data_clip (data/utils.py:57-70): preprocess_image with the processor returned by
    create_model_and_transforms (eval_clip.py:21-24).  A DeviceImageProcessor takes a list in one
    batched launch; any other callable is applied per image and stacked, as the reference does."""

    def __init__(self, image_processor):
        self.val_transform = image_processor

    def preprocess_image(self, image):
        if isinstance(image, list) and not isinstance(self.val_transform, DeviceImageProcessor):
            return torch.stack([self.val_transform(img) for img in image])
        return self.val_transform(image)
