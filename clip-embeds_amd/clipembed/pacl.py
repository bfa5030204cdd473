"""PACL / SPARC heads on top of the engine — mirrors Patch-Aligned-Contrastive-Learning/model/pacl.py.

Class names and forward signatures follow the reference so eval drivers read the same:
  open_clip_pacl            pacl.py:51-145  (forward: ones-weighted patch sum, "Eval only" overwrite :142)
  open_clip_pacl_rope       pacl.py:184-197 (RoPE on the 1024-d patch tokens before the head)
  open_clip_pacl_rope_after pacl.py:199-209 (RoPE on projected tokens, sigmoid(10 cos) weights)
  sparc                     pacl.py:380-478 (forward / scoring / forward_text mask)
  sparc_rope                pacl.py:480-484 (RoPE on the patch tokens before the visual head)
  apply_rope                pacl.py:147-181
  ClipLoss, SparcLoss       pacl.py:486-584 (temperature-scaled CLIP loss; SPARC global + masked local)
Everything runs through libclipembed; the fused pooling is ce_pacl_pool.
"""
from __future__ import annotations

import torch

from . import _lib
from .config import get_model_config
from .model import CLIP, _ptr, _stream, kernel_engine
from .weights import synthetic_pacl_heads


class open_clip_pacl(torch.nn.Module):
    weight_mode = _lib.CE_PACL_ONES
    rope = _lib.CE_ROPE_NONE

    def __init__(self, base_model: str = "ViT-L-14-336", clip_state_dict=None, device=None, cfg=None):
        super().__init__()
        if cfg is None:
            if base_model != "ViT-L-14-336":
                raise NotImplementedError(f"clipembed implements the ViT-L-14-336 PACL head only, not {base_model}")
            cfg = get_model_config(base_model)
        cfg = cfg.with_pacl(768)
        self.clip_model = CLIP(cfg)
        self.clip_model.visual.output_tokens = True          # pacl.py:100
        if clip_state_dict is not None:
            self.clip_model.load_state_dict(clip_state_dict)
        self._heads = {}
        if device is not None:
            self.to(device)

    # state dict with the reference's key layout: clip_model.* + visual_projection.* + text_projection.*
    def load_state_dict(self, sd, strict: bool = True):
        clip, heads = {}, {}
        for k, v in sd.items():
            k2 = k[7:] if k.startswith("module.") else k        # eval_pacl.py:380-388
            if k2.startswith("clip_model."):
                clip[k2[len("clip_model."):]] = v
            else:
                heads[k2] = v
        if clip:
            self.clip_model.load_state_dict(clip, strict=strict)
        if heads:
            self._heads.update(heads)
            if self.clip_model._engine is not None:
                self.clip_model._engine.load(heads, allow_unknown=not strict)
        return self

    def init_synthetic_heads(self, seed: int = 11):
        return self.load_state_dict(synthetic_pacl_heads(self.clip_model.cfg, seed))

    def to(self, *args, **kwargs):
        self.clip_model.to(*args, **kwargs)
        if self._heads and self.clip_model._engine is not None:
            self.clip_model._engine.load(self._heads, allow_unknown=True)
        return self

    @property
    def engine(self):
        return self.clip_model.engine

    @torch.no_grad()
    def forward_visual(self, images):
        """visual_projection(encode_image tokens) -> [B, 576, 768] (pacl.py:112-114)."""
        e = self.engine
        _, tokens = self.clip_model.encode_image(images)
        if self.rope == _lib.CE_ROPE_BEFORE:
            tokens = apply_rope(tokens, engine=e)
        B, P, _ = tokens.shape
        out = torch.empty(B, P, self.clip_model.cfg.pacl_dim, device=e.device, dtype=torch.float32)
        _lib.call("ce_pacl_project_patches", e.h, _stream(e.device), _ptr(tokens), _lib.CE_F32, B, P,
                  _lib.CE_ROPE_NONE, _ptr(out), _lib.CE_F32)
        return out

    @torch.no_grad()
    def forward_text(self, caps):
        """text_projection(encode_text) -> [B, 768] (pacl.py:116-118)."""
        e = self.engine
        t = self.clip_model.encode_text(caps)
        out = torch.empty(t.shape[0], self.clip_model.cfg.pacl_dim, device=e.device, dtype=torch.float32)
        _lib.call("ce_pacl_project_text", e.h, _stream(e.device), _ptr(t), t.shape[0], _ptr(out))
        return out

    @torch.no_grad()
    def pool(self, visual_proj, text_proj):
        """Fused patch alignment + weighted patch sum + L2 norms (pacl.py:120-145)."""
        e = self.engine
        vp = visual_proj.contiguous()
        tp = text_proj.float().contiguous()
        Bi, P, D = vp.shape
        Bt = tp.shape[0]
        R = max(Bi, Bt)
        oi = torch.empty(R, D, device=e.device, dtype=torch.float32)
        ot = torch.empty(Bt, D, device=e.device, dtype=torch.float32)
        dt = _lib.CE_BF16 if vp.dtype == torch.bfloat16 else _lib.CE_F32
        _lib.call("ce_pacl_pool", e.h, _stream(e.device), _ptr(vp), dt, Bi, P, _ptr(tp), Bt, D,
                  self.weight_mode, 1 if self.rope == _lib.CE_ROPE_AFTER else 0, _ptr(oi), _ptr(ot))
        return oi, ot

    @torch.no_grad()
    def forward(self, images, caps):
        """Whole PACL forward in one engine call (pacl.py:135-145 and the rope variants)."""
        e = self.engine
        images = self.clip_model._in(images, (torch.float32, torch.bfloat16))
        caps = self.clip_model._in(caps, (torch.int64,))
        Bi, Bt = images.shape[0], caps.shape[0]
        D = self.clip_model.cfg.pacl_dim
        oi = torch.empty(max(Bi, Bt), D, device=e.device, dtype=torch.float32)
        ot = torch.empty(Bt, D, device=e.device, dtype=torch.float32)
        pdt = _lib.CE_BF16 if images.dtype == torch.bfloat16 else _lib.CE_F32
        _lib.call("ce_pacl_forward", e.h, _stream(e.device), _ptr(images), pdt, Bi, _ptr(caps), Bt,
                  self.weight_mode, self.rope, _ptr(oi), _ptr(ot))
        return oi, ot


class open_clip_pacl_rope(open_clip_pacl):
    rope = _lib.CE_ROPE_BEFORE


class open_clip_pacl_rope_after(open_clip_pacl):
    weight_mode = _lib.CE_PACL_SIGMOID10
    rope = _lib.CE_ROPE_AFTER


class open_clip_pacl_sigmoid(open_clip_pacl):
    """sigmoid(10 cos) weighting without RoPE (the reference's *_base weighting, pacl.py:362-363)."""
    weight_mode = _lib.CE_PACL_SIGMOID10


@torch.no_grad()
def apply_rope(embeddings: torch.Tensor, engine=None) -> torch.Tensor:
    """apply_rope (pacl.py:147-181) on device; positions 0..P-1, de-interleaved output."""
    if engine is None:
        raise RuntimeError("apply_rope needs an engine (its RoPE tables live on the device)")
    x = embeddings.float().contiguous()
    B, P, D = x.shape
    out = torch.empty_like(x)
    _lib.call("ce_apply_rope", engine.h, _stream(engine.device), _ptr(x), B, P, D, _ptr(out))
    return out


class sparc(open_clip_pacl):
    """SPARC (pacl.py:380-478) on the ViT-L-14-336 head."""

    def __init__(self, sigma: float = 1.0 / 625, base_model: str = "ViT-L-14-336", **kw):
        super().__init__(base_model, **kw)
        self.sigma = sigma
        self.clip_model.output_text_tokens = True            # pacl.py:416

    @torch.no_grad()
    def forward_text(self, caps):
        e = self.engine
        caps = self.clip_model._in(caps, (torch.int64,))
        _, tokens = self.clip_model.encode_text(caps)
        B, T, Dt = tokens.shape
        D = self.clip_model.cfg.pacl_dim
        out = torch.empty(B, T, D, device=e.device, dtype=torch.float32)
        _lib.call("ce_pacl_project_text", e.h, _stream(e.device), _ptr(tokens), B * T, _ptr(out))
        eots = caps.argmax(dim=-1)
        mask = (torch.arange(T, device=caps.device).expand(B, -1) <= eots.unsqueeze(1)).float()
        return out, mask

    @torch.no_grad()
    def align(self, v_patch_embed, l_token_embed):
        """The similarity / min-max / threshold / alignment-weighting / grouping / L2 steps of
        sparc.forward (pacl.py:455-476) on given patch [B,P,D] and token [B,T,D] embeddings (also the
        train_sparc.py path with precomputed text embeddings).  Returns (grouped_normalised,
        tokens_normalised)."""
        e = self.engine
        v = v_patch_embed.float().contiguous()
        l = l_token_embed.float().contiguous()
        B, P, D = v.shape
        T = l.shape[1]
        if l.shape[0] != B or l.shape[2] != D:
            raise ValueError(f"sparc: patch {tuple(v.shape)} and token {tuple(l.shape)} embeddings do not match")
        grouped = torch.empty(B, T, D, device=e.device, dtype=torch.float32)
        l_norm = torch.empty_like(grouped)
        _lib.call("ce_sparc_forward", e.h, _stream(e.device), _ptr(v), _ptr(l), B, P, T, D, float(self.sigma),
                  _ptr(grouped), _ptr(l_norm), None)
        return grouped, l_norm

    @torch.no_grad()
    def forward(self, images, caps):
        v = self.forward_visual(images)
        l, mask = self.forward_text(caps)
        grouped, l_norm = self.align(v, l)
        return v, l_norm, grouped, mask

    @torch.no_grad()
    def scoring(self, images, caps, local: bool = False):
        if images.shape[0] == 1 and caps.shape[0] > 1:
            images = images.expand(caps.shape[0], *images.shape[1:])
        assert images.shape[0] == caps.shape[0]
        v, l, g, _ = self.forward(images, caps)
        gt = torch.nn.functional.normalize(l.mean(dim=1), dim=-1)
        if not local:
            gi = torch.nn.functional.normalize(v.mean(dim=1), dim=-1)
        else:
            gi = torch.nn.functional.normalize(g.mean(dim=1), dim=-1)
        return self.clip_model.logits(gi, gt, 1.0, with_text_logits=False)[0]


class sparc_rope(sparc):
    """sparc_rope (pacl.py:480-484): apply_rope on the 1024-d patch tokens before the visual head."""
    rope = _lib.CE_ROPE_BEFORE


def _all_gather_rows(x: torch.Tensor, world_size: int, rank: int):
    """Every rank's [B_r, D] rows concatenated in rank order, and this rank's first row in it
    (torch.distributed: RCCL over xGMI with the "nccl" backend; gloo in the CPU / single-GPU tests).
    The ranks may hold different B_r (an uneven last batch; nn.DataParallel's scatter splits unevenly
    too): the sizes are gathered first and the rows padded to the largest, as open_clip's
    gather_features_diffsize does (loss.py:67-87)."""
    import torch.distributed as dist
    x = x.contiguous()
    n = torch.tensor([x.shape[0]], device=x.device, dtype=torch.int64)
    sizes = [torch.empty_like(n) for _ in range(world_size)]
    dist.all_gather(sizes, n)
    sizes = [int(s) for s in sizes]
    mx = max(sizes)
    if all(s == mx for s in sizes):
        parts = [torch.empty_like(x) for _ in range(world_size)]
        dist.all_gather(parts, x)
    else:
        pad = torch.zeros((mx,) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        pad[:x.shape[0]] = x
        parts = [torch.empty_like(pad) for _ in range(world_size)]
        dist.all_gather(parts, pad)
        parts = [p[:s] for p, s in zip(parts, sizes)]
    return torch.cat(parts, dim=0), sum(sizes[:rank])


def _value_only(name: str, *tensors):
    """The engine's losses return the reference's VALUE (logging, evaluation): no autograd runs through
    the engine (nor through the sharded path's all-gather), so a caller that needs gradients must not
    get a silently detached loss.  Training goes through the trainers, which compute the gradients in
    the engine: clipembed.SparcHeadTrainer (train_sparc.py's step), clipembed.TextTowerTrainer (NegCLIP)."""
    if torch.is_grad_enabled() and any(t.requires_grad for t in tensors):
        raise RuntimeError(f"{name} returns the loss value only (no autograd through the engine); call it under "
                           "torch.no_grad() or on detached inputs, and train with clipembed.SparcHeadTrainer / "
                           "TextTowerTrainer")


def _all_reduce_sum(x: torch.Tensor) -> torch.Tensor:
    import torch.distributed as dist
    dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x


class ClipLoss(torch.nn.Module):
    """PACL ClipLoss (pacl.py:486-514): logit_scale = 1 / temperature, labels arange, mean of the
    image->text and text->image cross entropies.  Logits and CE run in libclipembed.

    rank / world_size (not in the reference's signature, whose callers are single-process): the
    batch is sharded over data-parallel ranks, and the value is the reference's loss over the WHOLE
    batch, as train_pacl.py:34-36,95 computes it after nn.DataParallel gathers every replica's
    outputs to one device.  The ranks all-gather the [B_r, D] features (B_r may differ per rank:
    sizes first, padded rows), each takes the CE sums of its own rows of the global logits both ways
    (ce_contrastive_loss_partial), one all-reduce adds them, ce_loss_combine divides by the global
    batch.  Every rank returns the same value.  Both paths return the VALUE only (the engine runs no
    autograd, nor does the all-gather): with inputs that require grad they raise instead of returning
    a detached loss (_value_only; gradients: clipembed.SparcHeadTrainer / TextTowerTrainer)."""

    def __init__(self, temperature: float, engine=None, rank: int = 0, world_size: int = 1):
        super().__init__()
        self.logit_scale = 1.0 / temperature
        self.engine = engine
        self.rank = rank
        self.world_size = world_size

    def _engine(self, t: torch.Tensor):
        return self.engine if self.engine is not None else kernel_engine(t.device)

    def get_ground_truth(self, device, num_logits: int) -> torch.Tensor:
        return torch.arange(num_logits, device=device, dtype=torch.long)

    @torch.no_grad()
    def get_logits(self, image_features, text_features):
        e = self._engine(image_features)
        a = image_features.float().contiguous()
        b = text_features.float().contiguous()
        lpi = torch.empty(a.shape[0], b.shape[0], device=a.device, dtype=torch.float32)
        lpt = torch.empty(b.shape[0], a.shape[0], device=a.device, dtype=torch.float32)
        _lib.call("ce_get_logits", e.h, _stream(e.device), _ptr(a), a.shape[0], _ptr(b), b.shape[0], a.shape[1],
                  float(self.logit_scale), 0, _ptr(lpi), _ptr(lpt))
        return lpi, lpt

    def _ce(self, e, logits, labels):
        out = torch.empty((), device=logits.device, dtype=torch.float32)
        _lib.call("ce_cross_entropy", e.h, _stream(e.device), _ptr(logits), logits.shape[0], logits.shape[1],
                  _ptr(labels), _ptr(out))
        return out

    # --- the engine calls of the sharded path (a CPU test double replaces them in tests/test_dist_gloo.py)
    def _contrastive_parts(self, e, img_all, txt_all, row0, B):
        parts = torch.empty(5, device=img_all.device, dtype=torch.float32)
        _lib.call("ce_contrastive_loss_partial", e.h, _stream(e.device), _ptr(img_all), _ptr(txt_all),
                  img_all.shape[0], row0, B, img_all.shape[1], float(self.logit_scale), _ptr(parts))
        return parts

    def _combine(self, e, parts, n_global, global_weight, local_weight):
        out = torch.empty((), device=parts.device, dtype=torch.float32)
        _lib.call("ce_loss_combine", e.h, _stream(e.device), _ptr(parts), n_global, float(global_weight),
                  float(local_weight), _ptr(out))
        return out

    def forward(self, image_features, text_features):
        _value_only("ClipLoss", image_features, text_features)
        with torch.no_grad():
            return self._forward(image_features, text_features)

    def _forward(self, image_features, text_features):
        e = self._engine(image_features)
        if self.world_size > 1:
            a = image_features.float().contiguous()
            b = text_features.float().contiguous()
            B = a.shape[0]
            if b.shape[0] != B:
                raise ValueError(f"ClipLoss: {B} image rows but {b.shape[0]} text rows")
            img_all, row0 = _all_gather_rows(a, self.world_size, self.rank)
            txt_all, _ = _all_gather_rows(b, self.world_size, self.rank)
            parts = _all_reduce_sum(self._contrastive_parts(e, img_all, txt_all, row0, B))
            return self._combine(e, parts, img_all.shape[0], 1.0, 0.0)
        lpi, lpt = self.get_logits(image_features, text_features)
        labels = self.get_ground_truth(image_features.device, lpi.shape[0])
        return (self._ce(e, lpi, labels) + self._ce(e, lpt, labels)) / 2


class SparcLoss(ClipLoss):
    """SparcLoss (pacl.py:516-584): global_weight * CLIP loss of the normalised patch / token means
    + local_weight * the mean of the two masked pairwise local losses — one ce_sparc_loss call.

    rank / world_size: the reference's global-batch value (train_sparc.py:93,105: nn.DataParallel
    gathers the replicas' outputs, SparcLoss runs on the whole batch) from a batch sharded over
    ranks: ce_sparc_loss_means -> all-gather of the [B, 768] normalised means -> each rank's rows of
    the global CE both ways + its samples' masked local sums (ce_sparc_loss_partial) -> all-reduce of
    the 5 partial sums -> ce_loss_combine.  The local term stays per sample; only its sums and the
    mask count cross ranks.  Every rank returns the same value."""

    def __init__(self, temperature: float, engine=None, rank: int = 0, world_size: int = 1):
        super().__init__(temperature, engine, rank, world_size)
        self.global_weight = 0.5
        self.local_weight = 1.0

    def _means(self, e, v, lt):
        B, P, D = v.shape
        gi = torch.empty(B, D, device=v.device, dtype=torch.float32)
        gt = torch.empty_like(gi)
        _lib.call("ce_sparc_loss_means", e.h, _stream(e.device), _ptr(v), _ptr(lt), B, P, lt.shape[1], D,
                  _ptr(gi), _ptr(gt))
        return gi, gt

    def _sparc_parts(self, e, img_all, txt_all, row0, lt, g, m):
        B, T, D = lt.shape
        parts = torch.empty(5, device=lt.device, dtype=torch.float32)
        _lib.call("ce_sparc_loss_partial", e.h, _stream(e.device), _ptr(img_all), _ptr(txt_all), img_all.shape[0],
                  row0, _ptr(lt), _ptr(g), _ptr(m), B, T, D, 1.0 / float(self.logit_scale), _ptr(parts))
        return parts

    def forward(self, v_patch_embed, l_token_embed, l_grouped_v_patch_embed, language_mask):
        _value_only("SparcLoss", v_patch_embed, l_token_embed, l_grouped_v_patch_embed)
        with torch.no_grad():
            return self._forward(v_patch_embed, l_token_embed, l_grouped_v_patch_embed, language_mask)

    def _forward(self, v_patch_embed, l_token_embed, l_grouped_v_patch_embed, language_mask):
        e = self._engine(v_patch_embed)
        v = v_patch_embed.float().contiguous()
        lt = l_token_embed.float().contiguous()
        g = l_grouped_v_patch_embed.float().contiguous()
        m = language_mask.float().contiguous()
        B, P, D = v.shape
        T = lt.shape[1]
        if lt.shape != (B, T, D) or g.shape != (B, T, D) or m.shape != (B, T):
            raise ValueError(f"SparcLoss: shape mismatch v {tuple(v.shape)} l {tuple(lt.shape)} "
                             f"g {tuple(g.shape)} mask {tuple(m.shape)}")
        if self.world_size > 1:
            gi, gt = self._means(e, v, lt)
            img_all, row0 = _all_gather_rows(gi, self.world_size, self.rank)
            txt_all, _ = _all_gather_rows(gt, self.world_size, self.rank)
            parts = _all_reduce_sum(self._sparc_parts(e, img_all, txt_all, row0, lt, g, m))
            return self._combine(e, parts, img_all.shape[0], self.global_weight, self.local_weight)
        out = torch.empty((), device=v.device, dtype=torch.float32)
        _lib.call("ce_sparc_loss", e.h, _stream(e.device), _ptr(v), _ptr(lt), _ptr(g), _ptr(m), B, P, T, D,
                  1.0 / float(self.logit_scale), float(self.global_weight), float(self.local_weight), _ptr(out))
        return out
