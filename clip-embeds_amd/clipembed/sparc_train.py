"""SPARC head training step (BASELINE configs[4]: the train_sparc.py path) on a frozen CLIP.

Mirrors one iteration of Patch-Aligned-Contrastive-Learning/train_sparc.py:13-37 with the model and
optimizer of train_sparc.py:90-106 (sparc_rope(sigma=1/576), SparcLoss(temperature=0.1),
torch.optim.Adam(lr=1e-4)):

  1. the frozen towers (pacl.py:408: requires_grad False): visual tokens (ln_post'd patches) and text
     tokens (ln_final'd, every position) from the engine's encoders;
  2. ce_sparc_train_forward: the heads in train mode — [apply_rope] -> LayerNorm -> Dropout(0.1) ->
     Patch_Projection for the patches, LayerNorm -> Dropout(0.1) -> Linear for the text tokens (or
     precomputed token embeddings, the "LLM embeddings" input of BASELINE configs[4]), and the alignment;
  3. SparcLoss over the whole batch: the normalised patch / token means (ce_sparc_loss_means), their
     RCCL all-gather across data-parallel ranks and an all-reduce of the mask count, then
     ce_sparc_train_loss_grad (the loss's partial sums + its gradient for this rank's samples), an
     all-reduce of the 5 partial sums and ce_loss_combine (the value);
  4. ce_sparc_train_backward: gradients of the 12 head tensors (flat f32 buffer), summed over ranks by
     one RCCL all-reduce — nn.DataParallel's semantics (train_sparc.py:93: the replicas' outputs are
     gathered, the loss is the global one, the replicas' gradients add up);
  5. Adam (ce_adamw with weight decay 0 is torch.optim.Adam) on the f32 masters, then the engine's
     compute copies of the heads are refreshed (ce_sparc_train_sync_weights).

Dropout masks come from a counter hash of (seed + step) over each element's index in the GLOBAL batch
(ce_sparc_train_forward's sample0 = this rank's first sample), not torch's RNG: N ranks draw the masks
of the single-device step on the concatenated batch.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import _lib
from .model import _ptr, _stream
from .pacl import _all_gather_rows, open_clip_pacl, sparc
from .train import _tensor_entry

HEAD_TENSORS = ["visual_projection.0.weight", "visual_projection.0.bias",
                "visual_projection.2.linear_projection.0.weight", "visual_projection.2.linear_projection.0.bias",
                "visual_projection.2.non_linear_projection.0.weight", "visual_projection.2.non_linear_projection.0.bias",
                "visual_projection.2.non_linear_projection.2.weight", "visual_projection.2.non_linear_projection.2.bias",
                "text_projection.0.weight", "text_projection.0.bias", "text_projection.2.weight", "text_projection.2.bias"]


class SparcHeadTrainer:
    """Owns the f32 masters, gradients and Adam state of a `sparc` / `sparc_rope` model's heads on the
    model's device, laid out in HEAD_TENSORS order in flat buffers."""

    def __init__(self, model: sparc, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, dropout: float = 0.1, temperature: float = 0.1, seed: int = 0,
                 rank: int = 0, world_size: int = 1):
        self._check_model(model)
        self.model = model
        self.e = model.engine
        self.dev = self.e.device
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.dropout, self.temperature = dropout, temperature
        self.global_weight, self.local_weight = self._loss_weights()
        self.seed, self.rank, self.world = seed, rank, world_size
        heads = model._heads
        missing = [n for n in HEAD_TENSORS if n not in heads]
        if missing:
            raise RuntimeError(f"SPARC head weights missing: {missing[:3]} (load_state_dict / init_synthetic_heads)")
        shapes = [tuple(torch.as_tensor(heads[n]).shape) for n in HEAD_TENSORS]
        sizes = [int(torch.Size(s).numel()) for s in shapes]
        self.n_total = sum(sizes)
        self.param = torch.empty(self.n_total, device=self.dev, dtype=torch.float32)
        self.grad = torch.zeros_like(self.param)
        self.exp_avg = torch.zeros_like(self.param)
        self.exp_avg_sq = torch.zeros_like(self.param)
        self.views: Dict[str, torch.Tensor] = {}
        self.gviews: Dict[str, torch.Tensor] = {}
        off = 0
        for n, shp, sz in zip(HEAD_TENSORS, shapes, sizes):
            self.param[off:off + sz].copy_(torch.as_tensor(heads[n]).float().reshape(-1).to(self.dev))
            self.views[n] = self.param[off:off + sz].view(shp)
            self.gviews[n] = self.grad[off:off + sz].view(shp)
            off += sz
        self._keep = []
        Pn = (_lib.Tensor * len(HEAD_TENSORS))()
        Gn = (_lib.Tensor * len(HEAD_TENSORS))()
        for i, n in enumerate(HEAD_TENSORS):
            b = n.encode()
            self._keep.append(b)
            Pn[i] = _tensor_entry(b, self.views[n])
            Gn[i] = _tensor_entry(b, self.gviews[n])
        _lib.call("ce_sparc_train_bind", self.e.h, Pn, Gn, len(HEAD_TENSORS))
        _lib.call("ce_sparc_train_sync_weights", self.e.h, _stream(self.dev))
        self.step_count = 0
        self.last_seed = None
        self.parts = torch.zeros(5, device=self.dev, dtype=torch.float32)

    # ------------------------------------------------------------------ model-specific pieces
    def _check_model(self, model):
        if not isinstance(model, sparc):
            raise TypeError("SparcHeadTrainer trains the heads of clipembed.pacl.sparc / sparc_rope")

    def _loss_weights(self):
        return 0.5, 1.0                                          # SparcLoss (pacl.py:519-521)

    def _text_input(self, caps, l_token_embed):
        """(text [B, T, E] f32, text_mode): the text tower's tokens through text_projection, or the
        precomputed token embeddings as they are."""
        m = self.model
        if caps is not None:
            caps = m.clip_model._in(caps, (torch.int64,))
            _, text = m.clip_model.encode_text(caps)
            return text, 0, caps
        return l_token_embed.to(self.dev).float(), 1, None

    def _default_mask(self, B, T):
        if self._caps is None:
            raise ValueError("SparcHeadTrainer: language_mask is required with l_token_embed")
        eots = self._caps.argmax(dim=-1)
        return (torch.arange(T, device=self.dev).expand(B, -1) <= eots.unsqueeze(1)).float()

    # ------------------------------------------------------------------ the step
    def forward(self, images: torch.Tensor, caps: Optional[torch.Tensor] = None,
                l_token_embed: Optional[torch.Tensor] = None, patch_tokens: Optional[torch.Tensor] = None):
        """Steps 1-2: frozen towers + the heads in train mode.  Returns (v, l, g) as sparc.forward does
        (pacl.py:453-478; l and g L2-normalised).  Exactly one of caps (text tower + text_projection) and
        l_token_embed ([B, T, 768] precomputed token embeddings) is given."""
        m = self.model
        if (caps is None) == (l_token_embed is None):
            raise ValueError("SparcHeadTrainer.forward: pass caps or l_token_embed (one of them)")
        if patch_tokens is None:
            _, patch_tokens = m.clip_model.encode_image(images)
        patch_tokens = patch_tokens.float().contiguous()
        text, mode, caps = self._text_input(caps, l_token_embed)
        text = text.contiguous()
        B, P, _ = patch_tokens.shape
        T = text.shape[1]
        Pd = m.clip_model.cfg.pacl_dim
        sample0 = 0
        if self.world > 1:                     # this rank's first sample in the global batch
            n = torch.tensor([B], device=self.dev, dtype=torch.int64)
            sizes = [torch.empty_like(n) for _ in range(self.world)]
            dist.all_gather(sizes, n)
            sample0 = int(sum(int(x) for x in sizes[:self.rank]))
        v = torch.empty(B, P, Pd, device=self.dev, dtype=torch.float32)
        l = torch.empty(B, T, Pd, device=self.dev, dtype=torch.float32)
        g = torch.empty(B, T, Pd, device=self.dev, dtype=torch.float32)
        self.last_seed = self.seed + self.step_count
        _lib.call("ce_sparc_train_forward", self.e.h, _stream(self.dev), _ptr(patch_tokens), B, P, m.rope, _ptr(text),
                  mode, T, float(getattr(m, "sigma", 1.0 / 576)), float(self.dropout), ctypes.c_uint64(self.last_seed), ctypes.c_int64(sample0),
                  _ptr(v), _ptr(l), _ptr(g))
        self._caps = caps
        return v, l, g

    def compute_grads(self, images: torch.Tensor, caps: Optional[torch.Tensor] = None,
                      l_token_embed: Optional[torch.Tensor] = None, language_mask: Optional[torch.Tensor] = None,
                      patch_tokens: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Steps 1-4.  Returns the global loss (device scalar, no host sync); gradients are in self.grad /
        self.gviews.  language_mask [B, T] defaults to arange(T) <= argmax(caps) (pacl.py:433-435)."""
        v, l, g = self.forward(images, caps, l_token_embed, patch_tokens)
        B, P, Pd = v.shape
        T = l.shape[1]
        if language_mask is None:
            language_mask = self._default_mask(B, T)
        mask = language_mask.to(self.dev).float().contiguous()
        gi = torch.empty(B, Pd, device=self.dev, dtype=torch.float32)
        gt = torch.empty_like(gi)
        _lib.call("ce_sparc_loss_means", self.e.h, _stream(self.dev), _ptr(v), _ptr(l), B, P, T, Pd, _ptr(gi), _ptr(gt))
        if self.world > 1:
            img_all, row0 = _all_gather_rows(gi, self.world, self.rank)
            txt_all, _ = _all_gather_rows(gt, self.world, self.rank)
            mt = mask.sum().reshape(1)
            dist.all_reduce(mt)
            mask_total = float(mt)
        else:
            img_all, txt_all, row0 = gi, gt, 0
            mask_total = float(mask.sum())
        _lib.call("ce_sparc_train_loss_grad", self.e.h, _stream(self.dev), _ptr(img_all), _ptr(txt_all),
                  img_all.shape[0], row0, _ptr(mask), mask_total, float(self.temperature), self.global_weight,
                  self.local_weight, _ptr(self.parts))
        _lib.call("ce_sparc_train_backward", self.e.h, _stream(self.dev))
        if self.world > 1:
            dist.all_reduce(self.parts)
            dist.all_reduce(self.grad)                 # nn.DataParallel: replica gradients add up
        loss = torch.empty((), device=self.dev, dtype=torch.float32)
        _lib.call("ce_loss_combine", self.e.h, _stream(self.dev), _ptr(self.parts), img_all.shape[0],
                  self.global_weight, self.local_weight, _ptr(loss))
        return loss

    def apply_update(self, lr: Optional[float] = None):
        """Step 5: torch.optim.Adam (= AdamW with weight decay 0) on the masters, engine copies refreshed."""
        lr = self.lr if lr is None else lr
        self.step_count += 1
        b1, b2 = self.betas
        s = _stream(self.dev)
        _lib.call("ce_adamw", s, _ptr(self.param), _ptr(self.grad), _ptr(self.exp_avg), _ptr(self.exp_avg_sq),
                  self.n_total, lr, b1, b2, self.eps, self.wd, self.step_count)
        _lib.call("ce_sparc_train_sync_weights", self.e.h, s)

    def step(self, images, caps=None, l_token_embed=None, language_mask=None, lr: Optional[float] = None) -> float:
        """One optimizer step (train_sparc.py:29-37); returns the loss."""
        loss = self.compute_grads(images, caps, l_token_embed, language_mask)
        self.apply_update(lr)
        return float(loss)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """The heads' current f32 masters under the reference's names (+ Patch_Projection's alias)."""
        out = {n: v.detach().cpu().clone() for n, v in self.views.items()}
        out["visual_projection.2.text_projection.0.weight"] = out["visual_projection.2.linear_projection.0.weight"]
        out["visual_projection.2.text_projection.0.bias"] = out["visual_projection.2.linear_projection.0.bias"]
        return out


class PaclHeadTrainer(SparcHeadTrainer):
    """PACL head training step (train_pacl.py:16-40,106-107: model(images, caps), ClipLoss(temperature=0.1),
    loss.backward(), torch.optim.Adam(lr=1e-4)) for open_clip_pacl / open_clip_pacl_rope on a frozen CLIP
    (the reference script's own llm2clip_pacl_rope needs network weights).  The same engine step as
    SparcHeadTrainer with the PACL forward restated in its terms:

      * image features: visual_projection of the (RoPE'd) patch tokens, summed over the patches with
        weight 1 (pacl.py:135-145, the ones overwrite) and L2-normalised = normalize(mean over patches),
        exactly SparcLoss's global image feature;
      * text features: text_projection of the pooled text embedding (pacl.py:116-118) = SPARC's text
        head on one token per caption (T = 1, mask 1), normalised;
      * ClipLoss(temperature) = SparcLoss's global term with global weight 1 and local weight 0
        (pacl.py:489-514 vs 516-584), so the alignment's gradient is zero and only the global term's
        gradient reaches the heads.

    open_clip_pacl_rope_after (sigmoid(10 cos) weights of the RoPE'd projections) is not on this path."""

    def _check_model(self, model):
        from . import _lib as L
        if isinstance(model, sparc) or not isinstance(model, open_clip_pacl):
            raise TypeError("PaclHeadTrainer trains the heads of clipembed.pacl.open_clip_pacl / open_clip_pacl_rope")
        if model.weight_mode != L.CE_PACL_ONES or model.rope == L.CE_ROPE_AFTER:
            raise NotImplementedError("PaclHeadTrainer: the sigmoid-weighted variants (open_clip_pacl_rope_after) "
                                      "are not on the training path")

    def _loss_weights(self):
        return 1.0, 0.0                                          # ClipLoss = the CLIP term alone

    def _text_input(self, caps, l_token_embed):
        if caps is None or l_token_embed is not None:
            raise ValueError("PaclHeadTrainer.forward: pass caps (the open_clip_pacl text path)")
        m = self.model
        caps = m.clip_model._in(caps, (torch.int64,))
        pooled = m.clip_model.encode_text(caps)                  # [B, 768] (pacl.py:116-118)
        return pooled.float().unsqueeze(1), 0, caps

    def _default_mask(self, B, T):
        return torch.ones(B, T, device=self.dev, dtype=torch.float32)
