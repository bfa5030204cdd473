"""Contrastive losses with the embedding exchange — mirrors open_clip/src/open_clip/loss.py.

ClipLoss(local_loss, gather_with_grad, rank, world_size, usehardtext) keeps the reference's
argument names and semantics (loss.py:89-193):
  * world_size > 1: all-gather image and text embeddings (gather_features, loss.py:21-65);
    with usehardtext the text batches may differ in size per rank: sizes are all-gathered
    first, texts padded to the max, gathered, unpadded, and reordered [originals of every
    rank, then hard negatives of every rank] (gather_features_diffsize :67-87, reorder :144-153).
  * local_loss: logits_per_image = s * I_local @ T_all^T, logits_per_text = s * T_local @ I_all^T,
    labels = arange(B) + B*rank; hard-text rows get label -100 (get_mixed_ground_truth :127-135).
  * loss = (CE(logits_per_image, labels_i) + CE(logits_per_text, labels_t)) / 2.
The exchange is torch.distributed (RCCL over xGMI with backend "nccl", gloo on CPU for tests);
logits and cross-entropy run in libclipembed (ce_get_logits, ce_cross_entropy).  Forward only.
bench.py's multi-GPU legs call exactly this exchange (ClipLoss.get_logits / __call__ with
local_loss=True), and tests/test_dist_gloo.py runs it on 2 gloo ranks against the reference.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from . import _lib
from .model import _ptr, _stream


def all_gather_cat(x: torch.Tensor, world_size: int) -> torch.Tensor:
    parts = [torch.empty_like(x) for _ in range(world_size)]
    dist.all_gather(parts, x.contiguous())
    return torch.cat(parts, dim=0)


def gather_features(image_features, text_features, world_size: int):
    """gather_features (loss.py:21-65) without autograd: cat of every rank's embeddings."""
    return all_gather_cat(image_features, world_size), all_gather_cat(text_features, world_size)


def gather_features_diffsize(image_features, text_features, world_size: int) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """gather_features_diffsize (loss.py:67-87): text batches of different sizes per rank."""
    all_image = all_gather_cat(image_features, world_size)
    size = torch.tensor([text_features.shape[0], text_features.shape[1]], device=text_features.device,
                        dtype=torch.int32)
    sizes = [torch.empty_like(size) for _ in range(world_size)]
    dist.all_gather(sizes, size)
    max_num = max(int(s[0]) for s in sizes)
    pad = torch.zeros(max_num - text_features.shape[0], text_features.shape[1], device=text_features.device,
                      dtype=text_features.dtype)
    padded = torch.cat([text_features, pad]).contiguous()
    parts = [torch.empty_like(padded) for _ in range(world_size)]
    dist.all_gather(parts, padded)
    return all_image, [p[: int(s[0])] for p, s in zip(parts, sizes)]


def mixed_ground_truth(device, num_images: int, num_texts: int, rank: int, world_size: int, local_loss: bool):
    """get_mixed_ground_truth (loss.py:127-135)."""
    li = torch.arange(num_images, device=device, dtype=torch.long)
    if world_size > 1 and local_loss:
        li = li + num_images * rank
    lt = torch.cat([li, -100 * torch.ones(num_texts - num_images, device=device, dtype=torch.long)])
    return li, lt


class ClipLoss:
    def __init__(self, local_loss: bool = False, gather_with_grad: bool = False, cache_labels: bool = False,
                 rank: int = 0, world_size: int = 1, use_horovod: bool = False, usehardtext: bool = False,
                 engine=None):
        if use_horovod:
            raise NotImplementedError("horovod is not supported; use torch.distributed (RCCL)")
        self.local_loss = local_loss
        self.gather_with_grad = gather_with_grad
        self.rank = rank
        self.world_size = world_size
        self.usehardtext = usehardtext
        self.engine = engine

    def _engine(self, t: torch.Tensor):
        if self.engine is None:
            from .model import kernel_engine
            self.engine = kernel_engine(t.device)
        return self.engine

    def _logits(self, a: torch.Tensor, b: torch.Tensor, scale: float) -> torch.Tensor:
        """s * a @ b^T (ce_get_logits)."""
        return self._logits_both(a, b, scale, transpose=False)[0]

    def _logits_both(self, a: torch.Tensor, b: torch.Tensor, scale: float, transpose: bool = True):
        """(s * a @ b^T, its transpose) from one fused ce_get_logits launch (model.py:306-309)."""
        e = self._engine(a)
        a = a.float().contiguous()
        b = b.float().contiguous()
        out = torch.empty(a.shape[0], b.shape[0], device=a.device, dtype=torch.float32)
        tout = torch.empty(b.shape[0], a.shape[0], device=a.device, dtype=torch.float32) if transpose else None
        _lib.call("ce_get_logits", e.h, _stream(e.device), _ptr(a), a.shape[0], _ptr(b), b.shape[0], a.shape[1],
                  float(scale), 0, _ptr(out), _ptr(tout))
        return out, tout

    def _ce(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        e = self._engine(logits)
        out = torch.empty((), device=logits.device, dtype=torch.float32)
        labels = labels.to(torch.int64).contiguous()
        _lib.call("ce_cross_entropy", e.h, _stream(e.device), _ptr(logits), logits.shape[0], logits.shape[1],
                  _ptr(labels), _ptr(out))
        return out

    def get_logits(self, image_features, text_features, logit_scale):
        scale = float(logit_scale)
        if self.world_size > 1:
            if not self.usehardtext:
                all_image, all_text = gather_features(image_features, text_features, self.world_size)
            else:
                all_image, text_list = gather_features_diffsize(image_features, text_features, self.world_size)
                per = image_features.shape[0]
                originals = [t[:per] for t in text_list]
                hard = [t[per:] for t in text_list]
                all_text = torch.cat(originals + hard, dim=0)
            if self.local_loss:
                return self._logits(image_features, all_text, scale), self._logits(text_features, all_image, scale)
            return self._logits_both(all_image, all_text, scale)
        return self._logits_both(image_features, text_features, scale)

    @torch.no_grad()
    def __call__(self, image_features, text_features, logit_scale, output_dict: bool = False):
        dev = image_features.device
        lpi, lpt = self.get_logits(image_features, text_features, logit_scale)
        if self.usehardtext:
            li, lt = mixed_ground_truth(dev, lpi.shape[0], lpt.shape[0], self.rank, self.world_size, self.local_loss)
        else:
            li = torch.arange(lpi.shape[0], device=dev, dtype=torch.long)
            if self.world_size > 1 and self.local_loss:
                li = li + lpi.shape[0] * self.rank
            lt = li
        loss = (self._ce(lpi, li) + self._ce(lpt, lt)) / 2
        return {"contrastive_loss": loss} if output_dict else loss

    forward = __call__
