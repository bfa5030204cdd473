"""Model geometry registry (mirrors open_clip/src/open_clip/model_configs/*.json).

Only the ViT/text-transformer CLIP family on the hot path is registered: ViT-L-14-336 (the
north-star model, `model_configs/ViT-L-14-336.json`) and its QuickGELU twin.  Heads follow
open_clip's defaults: vision heads = width // head_width (64, model.py:30), mlp = 4 * width
(mlp_ratio 4.0, model.py:31,67).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class VisionCfg:
    image_size: int = 336
    patch_size: int = 14
    width: int = 1024
    layers: int = 24
    heads: int = 16
    mlp_width: int = 4096

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def num_patches(self) -> int:
        return self.grid * self.grid

    @property
    def seq_len(self) -> int:
        return self.num_patches + 1


@dataclass(frozen=True)
class TextCfg:
    context_length: int = 77
    vocab_size: int = 49408
    width: int = 768
    heads: int = 12
    layers: int = 12
    mlp_width: int = 3072


@dataclass(frozen=True)
class ModelConfig:
    name: str = "ViT-L-14-336"
    embed_dim: int = 768
    vision: VisionCfg = field(default_factory=VisionCfg)
    text: TextCfg = field(default_factory=TextCfg)
    quick_gelu: bool = False
    pacl_dim: int = 0     # PACL head output (768 for open_clip_pacl('ViT-L-14-336'), pacl.py:70-79)

    def with_depth(self, vision_layers: int, text_layers: int) -> "ModelConfig":
        """Same widths, fewer blocks (reduced-depth parity configs)."""
        return dataclasses.replace(
            self,
            name=f"{self.name}-v{vision_layers}t{text_layers}",
            vision=dataclasses.replace(self.vision, layers=vision_layers),
            text=dataclasses.replace(self.text, layers=text_layers),
        )

    def with_pacl(self, pacl_dim: int = 768) -> "ModelConfig":
        return dataclasses.replace(self, pacl_dim=pacl_dim)

    def open_clip_dict(self) -> dict:
        """The open_clip model-config dict (for CLIP(**cfg) in the golden generator)."""
        return {
            "embed_dim": self.embed_dim,
            "quick_gelu": self.quick_gelu,
            "vision_cfg": {"image_size": self.vision.image_size, "layers": self.vision.layers,
                           "width": self.vision.width, "patch_size": self.vision.patch_size},
            "text_cfg": {"context_length": self.text.context_length, "vocab_size": self.text.vocab_size,
                         "width": self.text.width, "heads": self.text.heads, "layers": self.text.layers},
        }


_REGISTRY = {
    "ViT-L-14-336": ModelConfig(),
    "ViT-L-14-336-quickgelu": ModelConfig(name="ViT-L-14-336-quickgelu", quick_gelu=True),
}


def list_models():
    return sorted(_REGISTRY)


def get_model_config(name: str) -> ModelConfig:
    if name not in _REGISTRY:
        raise RuntimeError(f"Model config for {name} not found; available: {list_models()}")
    return _REGISTRY[name]
