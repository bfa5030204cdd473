"""clipembed — MI355X-native (gfx950) CLIP ViT-L/14-336 + PACL/SPARC embedding engine.

Drop-in for the open_clip / PACL surface used by lst627/CLIP-Embeds' eval and train drivers;
all compute runs in libclipembed.so (hand-written HIP kernels) behind a C ABI.
"""
from ._lib import ClipEmbedError, LIB_PATH, exported_symbols
from .config import ModelConfig, get_model_config, list_models
from .model import (CLIP, Engine, create_model, create_model_and_transforms, list_pretrained_tags_by_model,
                    load_checkpoint, load_checkpoint_file, load_state_dict, resize_pos_embed)
from .train import TextTowerTrainer
from .sparc_train import PaclHeadTrainer, SparcHeadTrainer
from .tokenizer import SimpleTokenizer, decode, get_tokenizer, tokenize
from .transforms import image_transform, prepare_data, prepare_data_clip
from .weights import (synthetic_captions, synthetic_images, synthetic_images_u8, synthetic_pacl_heads,
                      synthetic_state_dict)

__version__ = "0.1.0"

__all__ = [
    "CLIP", "Engine", "ClipEmbedError", "ModelConfig", "LIB_PATH", "create_model",
    "create_model_and_transforms", "exported_symbols", "get_model_config", "image_transform", "list_models",
    "list_pretrained_tags_by_model", "load_checkpoint", "load_checkpoint_file", "load_state_dict", "resize_pos_embed", "prepare_data", "prepare_data_clip", "synthetic_captions", "synthetic_images", "synthetic_images_u8",
    "synthetic_pacl_heads", "synthetic_state_dict", "SimpleTokenizer", "tokenize", "decode", "get_tokenizer",
    "TextTowerTrainer", "SparcHeadTrainer", "PaclHeadTrainer",
]
