"""CLIP BPE tokenizer: the reference's `SimpleTokenizer` surface over the C++ BPE in libclipembed.

Mirrors open_clip/src/open_clip/tokenizer.py:133-277 (`SimpleTokenizer`, `tokenize`, `decode`) and
factory.py:616 (`get_tokenizer`) with the same names and argument meaning.  Text cleaning is done
here exactly as tokenizer.py:66-130 does it (html.unescape twice, whitespace collapse, lower /
canonicalize); the pre-tokenizer regex, byte-level mapping and BPE merges run in C++
(csrc/tokenizer.cpp, `ce_tokenize`).

ftfy (tokenizer.py:67) is not installed in this environment; `basic_clean` applies ftfy.fix_text
only when ftfy is importable, otherwise the identity -- the same stub the golden fixtures were
generated with (tests/golden/make_golden_tokenizer.py).  For well-formed text fix_text is the
identity apart from Unicode NFC normalisation.

The merges file (bpe_simple_vocab_16e6.txt.gz, OpenAI's BPE vocabulary) is data, not code; it is
not redistributed here.  It is found at `bpe_path`, $CLIPEMBED_BPE_PATH, or inside an installed
open_clip package, in that order.
"""
from __future__ import annotations

import ctypes
import gzip
import html
import importlib.util
import os
import string
from typing import List, Optional, Union

import numpy as np
import torch

from . import _lib

DEFAULT_CONTEXT_LENGTH = 77   # tokenizer.py:23


def default_bpe() -> str:
    """Location of bpe_simple_vocab_16e6.txt.gz (tokenizer.py:26-28)."""
    env = os.environ.get("CLIPEMBED_BPE_PATH")
    if env:
        return env
    spec = importlib.util.find_spec("open_clip")
    if spec is not None and spec.submodule_search_locations:
        for d in spec.submodule_search_locations:
            p = os.path.join(d, "bpe_simple_vocab_16e6.txt.gz")
            if os.path.exists(p):
                return p
    raise FileNotFoundError(
        "bpe_simple_vocab_16e6.txt.gz not found: pass bpe_path=..., set CLIPEMBED_BPE_PATH, or install open_clip")


try:  # tokenizer.py:14
    import ftfy as _ftfy
except ImportError:  # not in this image
    _ftfy = None


def basic_clean(text: str) -> str:
    """tokenizer.py:66-69"""
    if _ftfy is not None:
        text = _ftfy.fix_text(text)
    text = html.unescape(html.unescape(text))
    return text.strip()


def whitespace_clean(text: str) -> str:
    """tokenizer.py:72-75"""
    return " ".join(text.split()).strip()


def canonicalize_text(text: str, *, keep_punctuation_exact_string: Optional[str] = None,
                      trans_punctuation: dict = str.maketrans("", "", string.punctuation)) -> str:
    """tokenizer.py:104-130"""
    text = text.replace("_", " ")
    if keep_punctuation_exact_string:
        text = keep_punctuation_exact_string.join(
            part.translate(trans_punctuation) for part in text.split(keep_punctuation_exact_string))
    else:
        text = text.translate(trans_punctuation)
    text = text.lower()
    text = " ".join(text.split())
    return text.strip()


_CLEAN = {
    "canonicalize": lambda x: canonicalize_text(basic_clean(x)),      # tokenizer.py:78-80
    "lower": lambda x: whitespace_clean(basic_clean(x)).lower(),      # tokenizer.py:83-85
    "whitespace": lambda x: whitespace_clean(basic_clean(x)),         # tokenizer.py:88-90
}


def get_clean_fn(type: str):
    """tokenizer.py:93-101"""
    if type not in _CLEAN:
        raise ValueError(f"Invalid clean function ({type}).")
    return _CLEAN[type]


class SimpleTokenizer:
    """tokenizer.py:133-265.  `reduction_mask` strategies (random/shuffle/syntax truncation used by
    some open_clip training configs) are outside this engine's scope and raise."""

    def __init__(self, bpe_path: Optional[str] = None, additional_special_tokens: Optional[List[str]] = None,
                 context_length: Optional[int] = DEFAULT_CONTEXT_LENGTH, clean: str = "lower",
                 reduction_mask: str = ""):
        if reduction_mask:
            raise NotImplementedError(f"reduction_mask={reduction_mask!r} is not supported")
        path = bpe_path or default_bpe()
        with gzip.open(path) as f:
            merges = f.read()
        specials = list(additional_special_tokens or [])
        arr = (ctypes.c_char_p * max(1, len(specials)))(*[s.encode() for s in specials])
        h = ctypes.c_void_p()
        L = _lib.lib()
        if L.ce_tokenizer_create(merges, len(merges), arr, len(specials), ctypes.byref(h)) != 0:
            raise _lib.ClipEmbedError(_lib.CE_ERR_INVALID, L.ce_tokenizer_last_error().decode())
        self._h = h
        self._lib = L
        sot, eot = ctypes.c_int32(), ctypes.c_int32()
        L.ce_tokenizer_special_ids(h, ctypes.byref(sot), ctypes.byref(eot))
        self.sot_token_id, self.eot_token_id = sot.value, eot.value
        self.all_special_ids = [self.sot_token_id, self.eot_token_id] + [
            self.eot_token_id + 1 + i for i in range(len(specials))]
        self.vocab_size = L.ce_tokenizer_vocab_size(h)
        self.context_length = context_length
        self.clean_fn = get_clean_fn(clean)
        self.reduction_fn = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.ce_tokenizer_destroy(h)
            self._h = None

    def encode(self, text: str) -> List[int]:
        """tokenizer.py:213-219: ids of the cleaned text, no SOT/EOT."""
        b = self.clean_fn(text).encode("utf-8")
        n = ctypes.c_int()
        self._check(self._lib.ce_tokenizer_encode(self._h, b, None, 0, ctypes.byref(n)))
        out = np.empty(max(1, n.value), dtype=np.int32)
        self._check(self._lib.ce_tokenizer_encode(self._h, b, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[: n.value].tolist()

    def decode(self, tokens) -> str:
        """tokenizer.py:221-224"""
        ids = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32).reshape(-1))
        n = ctypes.c_int()
        self._check(self._lib.ce_tokenizer_decode(self._h, ids.ctypes.data, ids.size, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._check(self._lib.ce_tokenizer_decode(self._h, ids.ctypes.data, ids.size, buf, n.value + 1,
                                                  ctypes.byref(n)))
        return buf.raw[: n.value].decode("utf-8")

    def __call__(self, texts: Union[str, List[str]], context_length: Optional[int] = None) -> torch.LongTensor:
        """tokenizer.py:226-265: [len(texts), context_length] int64."""
        if isinstance(texts, str):
            texts = [texts]
        context_length = context_length or self.context_length
        assert context_length, "Please set a valid context length"
        enc = [self.clean_fn(t).encode("utf-8") for t in texts]
        arr = (ctypes.c_char_p * max(1, len(enc)))(*enc)
        out = torch.zeros(len(enc), context_length, dtype=torch.long)
        if not enc:
            return out
        self._check(self._lib.ce_tokenize(self._h, arr, len(enc), context_length, ctypes.c_void_p(out.data_ptr())))
        return out

    def _check(self, rc: int):
        if rc != 0:
            raise _lib.ClipEmbedError(_lib.CE_ERR_INVALID, self._lib.ce_tokenizer_last_error().decode())


_tokenizer: Optional[SimpleTokenizer] = None


def _default() -> SimpleTokenizer:
    global _tokenizer
    if _tokenizer is None:   # tokenizer.py:268 builds it at import; here on first use
        _tokenizer = SimpleTokenizer()
    return _tokenizer


def tokenize(texts: Union[str, List[str]], context_length: int = DEFAULT_CONTEXT_LENGTH) -> torch.LongTensor:
    """tokenizer.py:276-277"""
    return _default()(texts, context_length=context_length)


def decode(output_ids: torch.Tensor) -> str:
    """tokenizer.py:271-273"""
    return _default().decode(output_ids.cpu().numpy())


def get_tokenizer(model_name: str = "", context_length: Optional[int] = None, **kwargs) -> SimpleTokenizer:
    """factory.py:616.  The reference's callers ask for 'ViT-L-14-336' (data/utils.py:60) and
    'ViT-B-16' (data/image_caption_data.py:46): both are OpenAI-BPE models with context 77, as is every
    model config this engine knows."""
    from .config import _REGISTRY
    if context_length is None:
        cfg = _REGISTRY.get(model_name)
        context_length = cfg.text.context_length if cfg is not None else DEFAULT_CONTEXT_LENGTH
    return SimpleTokenizer(context_length=context_length, **kwargs)
