"""`clipembed.CLIP` — drop-in for the object returned by open_clip.create_model_and_transforms.

Mirrors the surface the reference callers use:
  encode_image / encode_text / get_logits / forward   open_clip/src/open_clip/model.py:279-310,415-435
  model.visual.output_tokens (pacl.py:100), model.output_text_tokens (pacl.py:416, model.py:299-300)
  logit_scale, state_dict() / load_state_dict(), .to(device), .eval(), .parameters()
All compute runs in libclipembed (HIP, gfx950) through its C ABI; tensors cross the boundary
as device pointers on the caller's current stream.  There is no CPU path: calling an encoder
on a model that was never moved to a GPU raises.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .config import ModelConfig, get_model_config


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_TORCH_TO_CE = {torch.float32: _lib.CE_F32, torch.bfloat16: _lib.CE_BF16, torch.float16: _lib.CE_F16}


class Engine:
    """Owns one libclipembed handle on one device."""

    def __init__(self, cfg: ModelConfig, device_index: int):
        self.cfg = cfg
        self.device = torch.device("cuda", device_index)
        c = _lib.Config()
        c.embed_dim = cfg.embed_dim
        c.activation = _lib.CE_ACT_QUICK_GELU if cfg.quick_gelu else _lib.CE_ACT_GELU_ERF
        c.image_size = cfg.vision.image_size
        c.patch_size = cfg.vision.patch_size
        c.vision = _lib.TowerConfig(cfg.vision.width, cfg.vision.layers, cfg.vision.heads, cfg.vision.mlp_width)
        c.context_length = cfg.text.context_length
        c.vocab_size = cfg.text.vocab_size
        c.text = _lib.TowerConfig(cfg.text.width, cfg.text.layers, cfg.text.heads, cfg.text.mlp_width)
        c.pacl_dim = cfg.pacl_dim
        h = ctypes.c_void_p()
        _lib.call("ce_create", ctypes.byref(c), device_index, ctypes.byref(h))
        self.h = h
        self.timing = False

    def close(self):
        if self.h:
            _lib.lib().ce_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, sd: Dict[str, object], allow_unknown: bool = False):
        keep = []
        arr = (_lib.Tensor * max(1, len(sd)))()
        for i, (k, v) in enumerate(sd.items()):
            if isinstance(v, torch.Tensor):
                v = v.detach().to("cpu")
                if v.dtype == torch.bfloat16:
                    a = v.contiguous().view(torch.int16).numpy()
                    dt = _lib.CE_BF16
                elif v.dtype == torch.float16:
                    a = v.contiguous().view(torch.int16).numpy()
                    dt = _lib.CE_F16
                else:
                    a = v.float().contiguous().numpy()
                    dt = _lib.CE_F32
            else:
                a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
                dt = _lib.CE_F32
            keep.append(a)
            name = k.encode()
            keep.append(name)
            arr[i].name = name
            arr[i].data = a.ctypes.data_as(ctypes.c_void_p)
            arr[i].dtype = dt
            arr[i].ndim = a.ndim
            for d in range(min(4, a.ndim)):
                arr[i].shape[d] = a.shape[d]
        _lib.call("ce_load_weights", self.h, arr, len(sd), 1 if allow_unknown else 0)

    def missing(self):
        n = ctypes.c_int()
        first = ctypes.c_char_p()
        _lib.call("ce_missing_weights", self.h, ctypes.byref(n), ctypes.byref(first))
        return n.value, (first.value or b"").decode()

    def set_ln_fold(self, on: bool) -> bool:
        """Fold both towers' block LayerNorms into their GEMMs (default on); returns the previous
        setting.  Takes effect for weights already loaded in whole-block calls (ce_set_ln_fold)."""
        prev = ctypes.c_int()
        _lib.call("ce_set_ln_fold", self.h, 1 if on else 0, ctypes.byref(prev))
        return prev.value == 1

    def set_resid_hl(self, on: bool) -> bool:
        """Keep the folded image tower's residual stream as hi/lo bf16 planes inside the blocks
        (default on); returns the previous setting (ce_set_resid_hl)."""
        prev = ctypes.c_int()
        _lib.call("ce_set_resid_hl", self.h, 1 if on else 0, ctypes.byref(prev))
        return prev.value == 1

    def set_pooled_prune(self, on: bool) -> bool:
        """Run each tower's last block for the pooled rows only (CLS / EOT) when no tokens are
        requested (default on); returns the previous setting (ce_set_pooled_prune)."""
        prev = ctypes.c_int()
        _lib.call("ce_set_pooled_prune", self.h, 1 if on else 0, ctypes.byref(prev))
        return prev.value == 1

    # ---- timing (roofline reporting) ----
    def set_timing(self, on: bool, only: str = ""):
        """Bracket kernel launches with HIP events (all tags, or only the launches tagged `only`)."""
        _lib.call("ce_set_kernel_timing_filter", self.h, only.encode())
        _lib.call("ce_set_kernel_timing", self.h, 1 if on else 0)
        self.timing = bool(on)

    def kernel_stats(self):
        out = []
        i = 0
        L = _lib.lib()
        while True:
            name = ctypes.create_string_buffer(64)
            ms, n, fl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            rc = L.ce_kernel_stats(self.h, i, name, 64, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl),
                                   ctypes.byref(by))
            if rc != _lib.CE_OK:
                break
            out.append({"name": name.value.decode(), "ms": ms.value, "launches": n.value, "flops": fl.value,
                        "bytes": by.value})
            i += 1
        return out



_KERNEL_ENGINES: Dict[int, "Engine"] = {}


def kernel_engine(device) -> "Engine":
    """A weightless handle per device for the loss / head entry points that need no tower weights
    (ce_get_logits, ce_cross_entropy, ce_sparc_loss ...): lets the reference's loss classes keep
    their constructor signatures (pacl.py:489-521, open_clip loss.py:89-103)."""
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError(f"clipembed runs on the GPU only (got a tensor on {device})")
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _KERNEL_ENGINES:
        _KERNEL_ENGINES[idx] = Engine(get_model_config("ViT-L-14-336"), idx)
    return _KERNEL_ENGINES[idx]

class VisualTower:
    """Stands in for `model.visual` (attributes read or toggled by the reference callers)."""

    def __init__(self, cfg: ModelConfig):
        self.output_tokens = False
        self.image_size = (cfg.vision.image_size, cfg.vision.image_size)
        self.patch_size = (cfg.vision.patch_size, cfg.vision.patch_size)
        self.grid_size = (cfg.vision.grid, cfg.vision.grid)
        self.output_dim = cfg.embed_dim


class CLIP(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, output_dict: bool = False):
        super().__init__()
        self.cfg = cfg
        self.output_dict = output_dict
        self.visual = VisualTower(cfg)
        self.output_text_tokens = False
        self.context_length = cfg.text.context_length
        self.vocab_size = cfg.text.vocab_size
        self.logit_scale = torch.nn.Parameter(torch.tensor(math.log(1 / 0.07)))
        self.logit_bias = None
        self._sd: Dict[str, torch.Tensor] = {}
        self._engine: Optional[Engine] = None

    # ---------------------------------------------------------------- weights / device
    def load_state_dict(self, state_dict, strict: bool = True):
        sd = {}
        for k, v in state_dict.items():
            t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))
            sd[k] = t.detach().cpu()
        if "logit_scale" in sd:
            with torch.no_grad():
                self.logit_scale.copy_(sd["logit_scale"].reshape(()).float())
        self._sd.update(sd)
        if self._engine is not None:
            self._engine.load(sd, allow_unknown=not strict)
        return self

    def state_dict(self, *args, **kwargs):
        out = dict(self._sd)
        out["logit_scale"] = self.logit_scale.detach().cpu().clone()
        return out

    def to(self, *args, **kwargs):
        device = None
        for a in list(args) + [kwargs.get("device")]:
            if isinstance(a, (str, torch.device)):
                device = torch.device(a)
            elif isinstance(a, int):
                device = torch.device("cuda", a)
        super().to(*[a for a in args if not isinstance(a, (str, torch.device, int))],
                    **{k: v for k, v in kwargs.items() if k != "device"})
        if device is not None and device.type == "cuda":
            idx = device.index if device.index is not None else torch.cuda.current_device()
            if self._engine is None or self._engine.device.index != idx:
                self._engine = Engine(self.cfg, idx)
                if self._sd:
                    self._engine.load(self._sd)
            self.logit_scale.data = self.logit_scale.data.to(device)
        return self

    def cuda(self, device=None):
        return self.to(torch.device("cuda", device if device is not None else torch.cuda.current_device()))

    @property
    def engine(self) -> Engine:
        if self._engine is None:
            raise RuntimeError("clipembed runs only on a HIP device: call model.to('cuda') first")
        return self._engine

    @property
    def device(self):
        return self.engine.device

    def _in(self, t: torch.Tensor, dtypes) -> torch.Tensor:
        dev = self.engine.device
        if t.device != dev:
            t = t.to(dev)
        if t.dtype not in dtypes:
            t = t.to(dtypes[0])
        return t.contiguous()

    # ---------------------------------------------------------------- encoders
    @torch.no_grad()
    def encode_image(self, image: torch.Tensor, normalize: bool = False):
        e = self.engine
        image = self._in(image, (torch.float32, torch.bfloat16))
        v = self.cfg.vision
        if image.dim() != 4 or tuple(image.shape[1:]) != (3, v.image_size, v.image_size):
            raise RuntimeError(f"encode_image expects [B,3,{v.image_size},{v.image_size}], got {tuple(image.shape)}")
        B = image.shape[0]
        pooled = torch.empty(B, self.cfg.embed_dim, device=e.device, dtype=torch.float32)
        tokens = None
        if self.visual.output_tokens:
            tokens = torch.empty(B, v.num_patches, v.width, device=e.device, dtype=torch.float32)
        _lib.call("ce_encode_image", e.h, _stream(e.device), _ptr(image), _TORCH_TO_CE[image.dtype], B,
                  1 if normalize else 0, _ptr(pooled), _ptr(tokens), _lib.CE_F32)
        return (pooled, tokens) if self.visual.output_tokens else pooled

    @torch.no_grad()
    def encode_text(self, text: torch.Tensor, normalize: bool = False):
        e = self.engine
        text = self._in(text, (torch.int64,))
        t = self.cfg.text
        if text.dim() != 2 or text.shape[1] != t.context_length:
            raise RuntimeError(f"encode_text expects [B,{t.context_length}] token ids, got {tuple(text.shape)}")
        B = text.shape[0]
        pooled = torch.empty(B, self.cfg.embed_dim, device=e.device, dtype=torch.float32)
        tokens = None
        if self.output_text_tokens:
            tokens = torch.empty(B, t.context_length, t.width, device=e.device, dtype=torch.float32)
        _lib.call("ce_encode_text", e.h, _stream(e.device), _ptr(text), B, t.context_length,
                  1 if normalize else 0, _ptr(pooled), _ptr(tokens), _lib.CE_F32)
        return (pooled, tokens) if self.output_text_tokens else pooled

    @torch.no_grad()
    def logits(self, image_features: torch.Tensor, text_features: torch.Tensor, scale: float,
               normalize: bool = False, with_text_logits: bool = True):
        """scale * I @ T^T (+ its transpose) in one fused kernel (model.py:306-309)."""
        e = self.engine
        a = self._in(image_features, (torch.float32,))
        b = self._in(text_features, (torch.float32,))
        Bi, D = a.shape
        Bt = b.shape[0]
        il = torch.empty(Bi, Bt, device=e.device, dtype=torch.float32)
        tl = torch.empty(Bt, Bi, device=e.device, dtype=torch.float32) if with_text_logits else None
        _lib.call("ce_get_logits", e.h, _stream(e.device), _ptr(a), Bi, _ptr(b), Bt, D, float(scale),
                  1 if normalize else 0, _ptr(il), _ptr(tl))
        return il, tl

    def get_logits(self, image, text):
        image_features = self._pooled(self.encode_image(image, normalize=True))
        text_features = self._pooled(self.encode_text(text, normalize=True))
        return self.logits(image_features, text_features, float(self.logit_scale.detach().exp()))

    @staticmethod
    def _pooled(x):
        return x[0] if isinstance(x, tuple) else x

    def forward(self, image: Optional[torch.Tensor] = None, text: Optional[torch.Tensor] = None):
        image_features = self._pooled(self.encode_image(image, normalize=True)) if image is not None else None
        text_features = self._pooled(self.encode_text(text, normalize=True)) if text is not None else None
        if self.output_dict:
            return {"image_features": image_features, "text_features": text_features,
                    "logit_scale": self.logit_scale.exp()}
        return image_features, text_features, self.logit_scale.exp()


PRETRAINED_DIR_ENV = "CLIPEMBED_PRETRAINED_DIR"

# The pretrained tags of the registered configs (open_clip pretrained.py:308-313, _VITL14_336):
# where open_clip would download them from, which names the local copy may carry, and the tag's
# activation (quick_gelu), checked against the model config as factory.py:435-445 does.
_PRETRAINED = {
    ("ViT-L-14-336", "openai"): {
        "hf_hub": "timm/vit_large_patch14_clip_336.openai/",
        "url": "https://openaipublic.azureedge.net/clip/models/3035c92b350959924f9f00213499208652fc7ea050643e8b385c2dac08641f02/ViT-L-14-336px.pt",
        "quick_gelu": True,
    },
}


def list_pretrained_tags_by_model(model_name: str):
    """open_clip pretrained.list_pretrained_tags_by_model for the registered configs."""
    return [t for (m, t) in _PRETRAINED if m == model_name]


def pretrained_candidates(model_name: str, tag: str, root: str):
    """Local file names searched under $CLIPEMBED_PRETRAINED_DIR for (model, tag), in order: the
    Hugging Face hub layout open_clip downloads (`<repo basename>/open_clip_model.safetensors`, then
    `open_clip_pytorch_model.bin`: HF_SAFE_WEIGHTS_NAME / HF_WEIGHTS_NAME, constants.py:9-10,
    preferred in that order by pretrained.py:784-797), the same two names under `<model>/<tag>/`,
    a flat `<model>-<tag>.{safetensors,bin,pt}`, and the URL's file name (`ViT-L-14-336px.pt`)."""
    import os
    cfg = _PRETRAINED[(model_name, tag)]
    hub = cfg["hf_hub"].strip("/").split("/")[-1]
    names = []
    for d in (hub, os.path.join(model_name, tag)):
        names += [os.path.join(d, "open_clip_model.safetensors"), os.path.join(d, "open_clip_pytorch_model.bin")]
    names += [f"{model_name}-{tag}.{ext}" for ext in ("safetensors", "bin", "pt")]
    names.append(os.path.basename(cfg["url"]))
    return [os.path.join(root, n) for n in names]


def resolve_pretrained(model_name: str, pretrained: str, quick_gelu: bool = False) -> str:
    """The checkpoint file for `pretrained` (factory.py:390-419): an existing file path is used as
    is; a known tag (pretrained.py:308-313) resolves to a local copy under $CLIPEMBED_PRETRAINED_DIR
    (there is no download: the engine never touches the network), with a RuntimeError naming the
    variable when it is unset or holds no copy; anything else raises the reference's error."""
    import os
    import warnings
    if os.path.isfile(pretrained):
        return pretrained
    tag = pretrained.lower()
    if (model_name, tag) not in _PRETRAINED:
        raise RuntimeError(f"Pretrained value '{pretrained}' is not a known tag or valid file path "
                           f"(known tags for {model_name}: {list_pretrained_tags_by_model(model_name)})")
    root = os.environ.get(PRETRAINED_DIR_ENV)
    if not root:
        raise RuntimeError(f"pretrained='{pretrained}' for {model_name} needs a local copy of the weights: set "
                           f"{PRETRAINED_DIR_ENV} to the directory holding it (open_clip would download "
                           f"{_PRETRAINED[(model_name, tag)]['hf_hub']}; clipembed never downloads)")
    cands = pretrained_candidates(model_name, tag, root)
    for c in cands:
        if os.path.isfile(c):
            if _PRETRAINED[(model_name, tag)]["quick_gelu"] != quick_gelu:
                warnings.warn(f"QuickGELU mismatch between final model config (quick_gelu={quick_gelu}) and "
                              f"pretrained tag '{pretrained}' (quick_gelu={_PRETRAINED[(model_name, tag)]['quick_gelu']}).",
                              UserWarning)
            return c
    raise RuntimeError(f"pretrained='{pretrained}' for {model_name}: no checkpoint under {PRETRAINED_DIR_ENV}={root}; "
                       f"looked for {cands}")


def create_model(model_name: str = "ViT-L-14-336", pretrained: Optional[str] = None, device=None,
                 state_dict: Optional[dict] = None, output_dict: bool = False, **_ignored) -> CLIP:
    """open_clip.create_model equivalent (factory.py:241-613) for the registered CLIP configs.

    pretrained: None (weights must then be supplied via `state_dict`/load_state_dict), a path to a
    local open_clip state dict (.pt/.bin loaded with weights_only=True, or .safetensors), or a known
    tag ('openai'), resolved to a local file by resolve_pretrained ($CLIPEMBED_PRETRAINED_DIR).
    """
    cfg = get_model_config(model_name)
    model = CLIP(cfg, output_dict=output_dict)
    if pretrained:
        load_checkpoint(model, resolve_pretrained(model_name, pretrained, cfg.quick_gelu))
    if state_dict is not None:
        model.load_state_dict(state_dict)
    if device is not None:
        model.to(device)
    return model


def create_model_and_transforms(model_name: str = "ViT-L-14-336", pretrained: Optional[str] = None,
                                device=None, **kw):
    """Returns (model, preprocess_train, preprocess_val) like open_clip (factory.py:822-958), both
    transforms on the device (clipembed.transforms.image_transform): preprocess_val = Pillow-exact
    bicubic resize + center crop + normalise; preprocess_train = RandomResizedCrop(scale=(0.9, 1.0))
    with the box drawn from the host torch RNG and the bicubic resample on the device.  eval_clip.py
    takes the SECOND value (eval_clip.py:21-24), so its What'sUp / MMVP scores use the train one."""
    from .transforms import image_transform
    aug_cfg = kw.pop("aug_cfg", None)
    model = create_model(model_name, pretrained, device, **kw)
    S = model.cfg.vision.image_size
    return (model, image_transform(S, is_train=True, aug_cfg=aug_cfg, device=device),
            image_transform(S, is_train=False, device=device))


def load_state_dict(checkpoint_path: str, device="cpu", weights_only: bool = True) -> dict:
    """open_clip factory.load_state_dict (factory.py:143-168): .safetensors via safetensors, else
    torch.load (weights_only by default); a {'state_dict': ...} wrapper is unwrapped, a TorchScript
    module gives its state_dict minus input_resolution / context_length / vocab_size, and the
    'module.' prefix is stripped from every key when the FIRST key starts with 'module'."""
    if str(checkpoint_path).endswith(".safetensors"):
        from safetensors.torch import load_file
        checkpoint = load_file(checkpoint_path, device=device)
    else:
        checkpoint = torch.load(checkpoint_path, map_location=device, weights_only=weights_only)
    if isinstance(checkpoint, dict) and "state_dict" in checkpoint:
        state_dict = checkpoint["state_dict"]
    elif isinstance(checkpoint, torch.jit.ScriptModule):
        state_dict = checkpoint.state_dict()
        for key in ("input_resolution", "context_length", "vocab_size"):
            state_dict.pop(key, None)
    else:
        state_dict = checkpoint
    if next(iter(state_dict.items()))[0].startswith("module"):
        state_dict = {k[7:]: v for k, v in state_dict.items()}
    return state_dict


def resize_pos_embed(state_dict: dict, model: "CLIP", interpolation: str = "bicubic", antialias: bool = True):
    """open_clip resize_pos_embed (model.py:748-779): a checkpoint whose visual positional grid
    differs from the model's is resampled with the same torch op (bicubic, antialias, on the host,
    once at load time; 1 class token kept)."""
    import torch.nn.functional as F
    old = state_dict.get("visual.positional_embedding", None)
    if old is None:
        return
    old = torch.as_tensor(old)
    gh, gw = model.visual.grid_size
    if gh * gw + 1 == old.shape[0]:
        return
    tok, img = old[:1], old[1:]
    og = int(math.sqrt(len(img)))
    img = img.reshape(1, og, og, -1).permute(0, 3, 1, 2)
    img = F.interpolate(img.float(), size=(gh, gw), mode=interpolation, antialias=antialias, align_corners=False)
    img = img.permute(0, 2, 3, 1).reshape(1, gh * gw, -1)[0].to(old.dtype)
    state_dict["visual.positional_embedding"] = torch.cat([tok, img], dim=0)


def resize_text_pos_embed(state_dict: dict, model: "CLIP", interpolation: str = "linear", antialias: bool = False):
    """open_clip resize_text_pos_embed (model.py:782-812): text positional rows resampled to the
    model's context length."""
    import torch.nn.functional as F
    old = state_dict.get("positional_embedding", None)
    if old is None:
        return
    old = torch.as_tensor(old)
    num_pos, width = model.cfg.text.context_length, model.cfg.text.width
    if old.shape[1] != width:
        raise ValueError("text pos_embed width changed!")
    if old.shape[0] == num_pos:
        return
    x = old.reshape(1, old.shape[0], width).permute(0, 2, 1)
    x = F.interpolate(x.float(), size=num_pos, mode=interpolation, antialias=antialias, align_corners=False)
    state_dict["positional_embedding"] = x.permute(0, 2, 1)[0].to(old.dtype)


def load_checkpoint(model: "CLIP", checkpoint_path: str, strict: bool = True, weights_only: bool = True,
                    device="cpu"):
    """open_clip factory.load_checkpoint (factory.py:171-215) for the registered CLIP configs:
    load_state_dict, logit_scale reshaped to the model's (0-d) parameter, position embeddings
    resized, then model.load_state_dict.  (3rd-party converters and big_vision .npz weights are
    not on the path.)"""
    state_dict = load_state_dict(checkpoint_path, device=device, weights_only=weights_only)
    if "logit_scale" in state_dict and torch.as_tensor(state_dict["logit_scale"]).ndim != model.logit_scale.ndim:
        state_dict["logit_scale"] = torch.as_tensor(state_dict["logit_scale"]).reshape(model.logit_scale.shape)
    state_dict.pop("text.transformer.embeddings.position_ids", None)
    resize_pos_embed(state_dict, model)
    resize_text_pos_embed(state_dict, model)
    model.load_state_dict(state_dict, strict=strict)
    return model


def load_checkpoint_file(path: str) -> dict:
    """State dict of a local open_clip checkpoint (load_state_dict above)."""
    return load_state_dict(path)
