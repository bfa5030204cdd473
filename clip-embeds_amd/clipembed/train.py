"""Contrastive training step of the text tower with a locked image tower.

Mirrors one iteration of open_clip_train/train.py:85-189 as launched by
open_clip/src/train-clip.sh (`--lock-image --local-loss --gather-with-grad [--usehardtext]
--lr 5e-6 --wd 0.0`, ViT AdamW betas (0.9, 0.98), eps 1e-6, params.py:9), with one process per GPU:

  1. image features: the frozen image tower forward (main.py:271-275 lock_image_tower), normalised;
  2. text features: the text tower forward with saved activations (ce_text_forward_train);
  3. ClipLoss (loss.py:137-193): RCCL all-gather of image features, of text sizes + padded text
     features (gather_features_diffsize :67-87), reorder originals before hard negatives
     (:144-153), local-loss logits [B, sum T] and [T_local, W*B], labels arange + B*rank with -100
     for hard negatives (:127-135), loss = (CE_i + CE_t) / 2;
  4. backward of the loss to the features (ce_contrastive_grad); the all-gather's backward (sum of
     every rank's gradient of this rank's rows) is an RCCL reduce_scatter of d(all text features),
     laid out in the gather's padded per-rank chunks;
  5. text-tower backward into one flat f32 gradient buffer (ce_text_backward), DDP's gradient
     all-reduce (main.py:302) bucketed as DDP does: ce_text_backward_events records an event as each
     bucket of blocks (top-down) has its final gradients, and each bucket's all_reduce(SUM) runs on
     a side stream behind its event while the blocks below are still in their backward; the sum is
     divided by the world size once all buckets are in (`bucket_blocks` blocks per bucket, 0 = one
     all_reduce of the whole buffer after the backward);
  6. AdamW on the flat f32 masters, two groups as main.py:335-349 (gain/bias/ln/logit_scale
     without weight decay), then the engine's compute copies are refreshed from the masters
     (ce_train_sync_weights) and logit_scale is clamped to [0, ln 100] (train.py:189).

All arithmetic is in libclipembed; torch.distributed moves the bytes (RCCL over xGMI, or gloo in
the CPU tests).  Mixed precision is the engine's (bf16 GEMM operands, f32 accumulation, f32
masters/gradients), standing in for the reference's `--precision amp`.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import _lib
from .model import CLIP, _ptr, _stream


def _excluded(name: str, t: torch.Tensor) -> bool:
    """main.py:335: no weight decay for 1-d tensors, norms, biases and logit_scale."""
    return t.ndim < 2 or "bn" in name or "ln" in name or "bias" in name or "logit_scale" in name


def text_tensor_names(model: CLIP) -> List[str]:
    names = ["token_embedding.weight", "positional_embedding", "ln_final.weight", "ln_final.bias", "text_projection"]
    for l in range(model.cfg.text.layers):
        for n in ("ln_1.weight", "ln_1.bias", "attn.in_proj_weight", "attn.in_proj_bias", "attn.out_proj.weight",
                  "attn.out_proj.bias", "ln_2.weight", "ln_2.bias", "mlp.c_fc.weight", "mlp.c_fc.bias",
                  "mlp.c_proj.weight", "mlp.c_proj.bias"):
            names.append(f"transformer.resblocks.{l}.{n}")
    return names


def _tensor_entry(name: bytes, t: torch.Tensor) -> _lib.Tensor:
    e = _lib.Tensor()
    e.name = name
    e.data = ctypes.c_void_p(t.data_ptr())
    e.dtype = _lib.CE_F32
    e.ndim = t.dim()
    for d in range(t.dim()):
        e.shape[d] = t.shape[d]
    return e


def negclip_feature_grad(img: torch.Tensor, txt: torch.Tensor, scale: float, rank: int, world: int, cgrad):
    """ClipLoss(local_loss=True, gather_with_grad=True, usehardtext=T > B) forward and backward to
    this rank's text features (loss.py:67-87, 127-193).  img [B, E], txt [B + K, E] (originals
    first, then this rank's hard negatives; K may differ per rank), both L2-normalised.
    cgrad(a, b, scale, labels, inv_count, da, db, weight) accumulates one CE direction (the
    engine's ce_contrastive_grad; a torch double in the CPU tests).  Returns d loss / d txt."""
    B, T = img.shape[0], txt.shape[0]
    dev = txt.device
    dtxt = torch.zeros_like(txt)
    if world > 1:
        parts = [torch.empty_like(img) for _ in range(world)]
        dist.all_gather(parts, img.contiguous())
        all_img = torch.cat(parts)
        size = torch.tensor([T], device=dev, dtype=torch.int64)
        sizes = [torch.empty_like(size) for _ in range(world)]
        dist.all_gather(sizes, size)
        sizes = [int(x) for x in sizes]
        padded = torch.zeros(max(sizes), txt.shape[1], device=dev, dtype=txt.dtype)
        padded[:T] = txt
        tparts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(tparts, padded)
        # originals of every rank, then hard negatives of every rank (loss.py:144-153)
        all_txt = torch.cat([p[:B] for p in tparts] + [p[B:n] for p, n in zip(tparts, sizes)]).contiguous()
    else:
        all_img, all_txt = img, txt
    li = torch.arange(B, device=dev, dtype=torch.long) + (B * rank if world > 1 else 0)
    lt = torch.cat([li, torch.full((T - B,), -100, device=dev, dtype=torch.long)]) if T > B else li
    d_all_txt = torch.zeros_like(all_txt)
    cgrad(img, all_txt, scale, li, 1.0 / B, None, d_all_txt, 0.5)    # CE(logits_per_image, li)
    cgrad(txt, all_img, scale, lt, 1.0 / B, dtxt, None, 0.5)         # CE(logits_per_text, lt)
    if world > 1:
        # backward of the all-gather = reduce-scatter: lay the gradient out in the
        # gather's padded per-rank chunks [originals of rank r | its hard negatives | zeros], sum
        # over ranks and keep this rank's chunk — half the bytes of an all-reduce of the whole
        mx = max(sizes)
        dpad = torch.zeros(world, mx, txt.shape[1], device=dev, dtype=d_all_txt.dtype)
        oh = world * B
        for r, n in enumerate(sizes):
            dpad[r, :B] = d_all_txt[r * B:(r + 1) * B]
            if n > B:
                dpad[r, B:n] = d_all_txt[oh:oh + n - B]
            oh += n - B
        mine = torch.empty(mx, txt.shape[1], device=dev, dtype=d_all_txt.dtype)
        dist.reduce_scatter_tensor(mine, dpad.view(world * mx, -1))
        dtxt += mine[:T]
    else:
        dtxt += d_all_txt
    return dtxt


class TextTowerTrainer:
    """Owns the f32 masters, gradients and AdamW state of the text tower (+ logit_scale) on the
    model's device, laid out as [decay group | no-decay group | logit_scale] in flat buffers."""

    def __init__(self, model: CLIP, lr: float = 5e-6, betas=(0.9, 0.98), eps: float = 1e-6,
                 weight_decay: float = 0.0, local_loss: bool = True, gather_with_grad: bool = True,
                 usehardtext: bool = False, rank: int = 0, world_size: int = 1, bucket_blocks: int = 1):
        if world_size > 1 and not (local_loss and gather_with_grad):
            raise NotImplementedError("the engine implements the train-clip.sh setting: --local-loss --gather-with-grad")
        self.model = model
        self.e = model.engine
        self.dev = self.e.device
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.usehardtext = usehardtext
        self.rank, self.world = rank, world_size
        names = text_tensor_names(model)
        missing = [n for n in names if n not in model._sd]
        if missing:
            raise RuntimeError(f"text tower weights missing from the model's state dict: {missing[:3]}")
        decay = [n for n in names if not _excluded(n, model._sd[n])]
        nodecay = [n for n in names if _excluded(n, model._sd[n])]
        order = decay + nodecay
        sizes = [model._sd[n].numel() for n in order]
        self.n_decay = sum(sizes[: len(decay)])
        self.n_total = sum(sizes) + 1                       # + logit_scale (no-decay group, last)
        self.param = torch.empty(self.n_total, device=self.dev, dtype=torch.float32)
        self.grad = torch.zeros_like(self.param)
        self.exp_avg = torch.zeros_like(self.param)
        self.exp_avg_sq = torch.zeros_like(self.param)
        self.views: Dict[str, torch.Tensor] = {}
        self.gviews: Dict[str, torch.Tensor] = {}
        off = 0
        for n, sz in zip(order, sizes):
            shape = tuple(model._sd[n].shape)
            self.param[off:off + sz].copy_(model._sd[n].float().reshape(-1).to(self.dev))
            self.views[n] = self.param[off:off + sz].view(shape)
            self.gviews[n] = self.grad[off:off + sz].view(shape)
            off += sz
        self.param[off] = float(model.logit_scale.detach())
        self.step_count = 0
        self._keep = []
        P = (_lib.Tensor * len(order))()
        G = (_lib.Tensor * len(order))()
        for i, n in enumerate(order):
            b = n.encode()
            self._keep.append(b)
            P[i] = _tensor_entry(b, self.views[n])
            G[i] = _tensor_entry(b, self.gviews[n])
        _lib.call("ce_train_bind", self.e.h, P, G, len(order))
        _lib.call("ce_train_sync_weights", self.e.h, _stream(self.dev))
        self.lossbuf = torch.zeros(2, device=self.dev, dtype=torch.float32)
        self.overlap_text = False           # text forward beside the image forward (compute_grads)
        self._side = None
        self._ar_side = None
        self.bucket_blocks = bucket_blocks
        self._buckets = self._make_buckets(bucket_blocks) if world_size > 1 and bucket_blocks > 0 else None

    def _runs(self, names, extra=()):
        """Contiguous [lo, hi) element ranges of the flat gradient buffer covering `names` (+ extra)."""
        base = self.grad.storage_offset()
        iv = sorted([(self.gviews[n].storage_offset() - base, self.gviews[n].storage_offset() - base +
                      self.gviews[n].numel()) for n in names] + list(extra))
        runs = [list(iv[0])]
        for lo, hi in iv[1:]:
            if lo == runs[-1][1]:
                runs[-1][1] = hi
            else:
                runs.append([lo, hi])
        return [tuple(r) for r in runs]

    def _make_buckets(self, per: int):
        """[(event index or None, runs)] in the order the backward finishes them: the head (+ logit_scale),
        groups of `per` blocks top-down (event after the group's lowest block), the embeddings (end)."""
        nl = self.model.cfg.text.layers
        n = self.n_total
        out = [(0, self._runs(["ln_final.weight", "ln_final.bias", "text_projection"], [(n - 1, n)]))]
        blocks = list(range(nl - 1, -1, -1))
        for i in range(0, nl, per):
            grp = blocks[i:i + per]
            names = [nm for b in grp for nm in self.gviews if nm.startswith(f"transformer.resblocks.{b}.")]
            out.append((1 + (nl - 1 - grp[-1]), self._runs(names)))
        out.append((None, self._runs(["token_embedding.weight", "positional_embedding"])))
        covered = sum(hi - lo for _, runs in out for lo, hi in runs)
        if covered != n:
            raise RuntimeError(f"gradient buckets cover {covered} of {n} elements")
        return out

    # ------------------------------------------------------------------ pieces
    @property
    def logit_scale(self) -> torch.Tensor:
        return self.param[-1]

    def text_forward(self, texts: torch.Tensor) -> torch.Tensor:
        texts = texts.to(self.dev, torch.int64).contiguous()
        f = torch.empty(texts.shape[0], self.model.cfg.embed_dim, device=self.dev, dtype=torch.float32)
        _lib.call("ce_text_forward_train", self.e.h, _stream(self.dev), _ptr(texts), texts.shape[0], _ptr(f))
        return f

    def _cgrad(self, a, b, scale, labels, inv_count, da, db, weight):
        _lib.call("ce_contrastive_grad", self.e.h, _stream(self.dev), _ptr(a), a.shape[0], _ptr(b), b.shape[0],
                  a.shape[1], float(scale), _ptr(labels), float(weight), float(inv_count), _ptr(self.lossbuf),
                  _ptr(da), _ptr(db))

    def loss_and_feature_grad(self, img: torch.Tensor, txt: torch.Tensor, scale: float):
        """ClipLoss forward + backward to the local text features (loss.py:137-193)."""
        self.lossbuf.zero_()
        return negclip_feature_grad(img, txt, scale, self.rank, self.world, self._cgrad)

    # ------------------------------------------------------------------ the step
    def compute_grads(self, images: torch.Tensor, texts: torch.Tensor) -> torch.Tensor:
        """Steps 1-5: forward, ClipLoss, backward, gradient all-reduce.  Returns the local loss (device
        scalar, no host sync); gradients are in self.grad / self.gviews.

        The locked image tower and the text tower's forward are independent until the loss: with
        `overlap_text` the text forward runs on a side stream beside the image forward and the loss
        waits for both.  Off by default: at the C4 size both towers' GEMMs are persistent grids of
        one workgroup per CU, so they take turns rather than fill each other's gaps (NegCLIP 453.7 vs
        451.8 ms/step)."""
        if not self.overlap_text:
            img = self.model.encode_image(images, normalize=True)
            return self.compute_grads_from_features(img, texts)
        if self.e.timing:
            # one handle on two concurrent streams: its per-kernel event brackets and the profile
            # pass's host readbacks are not stream-aware, so timings would be misattributed
            raise RuntimeError("TextTowerTrainer.overlap_text cannot run with engine kernel timing on "
                               "(Engine.set_timing): turn one of them off")
        main = torch.cuda.current_stream(self.dev)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
        side = self._side
        texts = texts.to(self.dev, torch.int64).contiguous()
        side.wait_stream(main)                      # the caption ids (and the weights) are ready
        with torch.cuda.stream(side):
            txt = self.text_forward(texts)
        texts.record_stream(side)
        img = self.model.encode_image(images, normalize=True)
        main.wait_stream(side)
        txt.record_stream(main)
        return self._grads_from_text(img, txt)

    def compute_grads_from_features(self, img: torch.Tensor, texts: torch.Tensor) -> torch.Tensor:
        """Steps 2-5 given the locked image tower's normalised features img [B, E] (step 1)."""
        return self._grads_from_text(img, self.text_forward(texts))

    def _grads_from_text(self, img: torch.Tensor, txt: torch.Tensor) -> torch.Tensor:
        """Steps 3-5 given both towers' features (txt from ce_text_forward_train on this handle)."""
        scale = math.exp(float(self.logit_scale))
        dtxt = self.loss_and_feature_grad(img, txt, scale)
        if self.world > 1 and self._buckets is not None:
            self._backward_bucketed(dtxt, txt.shape[0])
            return self.lossbuf[0].clone()
        _lib.call("ce_text_backward", self.e.h, _stream(self.dev), _ptr(dtxt), txt.shape[0])
        self.grad[-1:].copy_(self.lossbuf[1:2])       # d loss / d logit_scale
        if self.world > 1:                            # DDP: average over ranks, one flat buffer
            dist.all_reduce(self.grad)
            self.grad.div_(self.world)
        return self.lossbuf[0].clone()

    def _backward_bucketed(self, dtxt: torch.Tensor, T: int):
        """Step 5 with DDP's overlap: bucket k's all_reduce is enqueued on a side stream behind the
        event the backward records when that bucket's gradients are final."""
        main = torch.cuda.current_stream(self.dev)
        if self._ar_side is None:
            self._ar_side = torch.cuda.Stream(device=self.dev)
            nl = self.model.cfg.text.layers
            self._events = [None] * (nl + 1)
            for ev_i, _ in self._buckets:
                if ev_i is not None:
                    ev = torch.cuda.Event()
                    ev.record(main)                   # creates the event (re-recorded by the engine)
                    self._events[ev_i] = ev
            self._ev_ptrs = (ctypes.c_void_p * (nl + 1))(
                *[ctypes.c_void_p(ev.cuda_event) if ev is not None else None for ev in self._events])
        side = self._ar_side
        self.grad[-1:].copy_(self.lossbuf[1:2])       # d loss / d logit_scale (the head bucket)
        _lib.call("ce_text_backward_events", self.e.h, _stream(self.dev), _ptr(dtxt), T, self._ev_ptrs,
                  len(self._ev_ptrs))
        works = []
        with torch.cuda.stream(side):
            for ev_i, runs in self._buckets:
                if ev_i is None:
                    side.wait_stream(main)            # the embeddings: the end of the backward
                else:
                    side.wait_event(self._events[ev_i])
                for lo, hi in runs:
                    works.append(dist.all_reduce(self.grad[lo:hi], async_op=True))
        for w in works:
            w.wait()                                  # the current (main) stream waits for the sums
        main.wait_stream(side)
        self.grad.div_(self.world)

    def apply_update(self, lr: Optional[float] = None):
        """Step 6: AdamW on both groups, logit_scale clamp, engine weights refreshed."""
        lr = self.lr if lr is None else lr
        self.step_count += 1
        b1, b2 = self.betas
        s = _stream(self.dev)
        _lib.call("ce_adamw", s, _ptr(self.param), _ptr(self.grad), _ptr(self.exp_avg), _ptr(self.exp_avg_sq),
                  self.n_decay, lr, b1, b2, self.eps, self.wd, self.step_count)
        rest = self.n_total - self.n_decay
        off = self.n_decay * 4
        _lib.call("ce_adamw", s, ctypes.c_void_p(self.param.data_ptr() + off),
                  ctypes.c_void_p(self.grad.data_ptr() + off), ctypes.c_void_p(self.exp_avg.data_ptr() + off),
                  ctypes.c_void_p(self.exp_avg_sq.data_ptr() + off), rest, lr, b1, b2, self.eps, 0.0, self.step_count)
        self.param[-1:].clamp_(0, math.log(100))      # train.py:189
        _lib.call("ce_train_sync_weights", self.e.h, s)
        with torch.no_grad():
            self.model.logit_scale.copy_(self.param[-1])

    def step(self, images: torch.Tensor, texts: torch.Tensor, lr: Optional[float] = None) -> float:
        """One optimizer step on (images [B,3,H,W], texts [B+K,77]); returns the local loss."""
        loss = self.compute_grads(images, texts)
        self.apply_update(lr)
        return float(loss)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """The text tower's current f32 masters (+ logit_scale), open_clip names."""
        out = {n: v.detach().cpu().clone() for n, v in self.views.items()}
        out["logit_scale"] = self.param[-1].detach().cpu().clone()
        return out
