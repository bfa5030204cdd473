"""C++ BPE tokenizer (csrc/tokenizer.cpp via clipembed.tokenizer) against golden ids produced by the
reference's own SimpleTokenizer (tests/golden/make_golden_tokenizer.py; ftfy stubbed to identity in
both).  Needs the BPE merges file (OpenAI data, not redistributed): $CLIPEMBED_BPE_PATH, an installed
open_clip, or the reference tree in the build container; skipped when none is present."""
import os

import numpy as np
import pytest
import torch

from clipembed import tokenizer as T

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "tokenizer.npz"))
_REF_BPE = "/root/reference/open_clip/src/open_clip/bpe_simple_vocab_16e6.txt.gz"


def _bpe():
    try:
        return T.default_bpe()
    except FileNotFoundError:
        if os.path.exists(_REF_BPE):
            return _REF_BPE
        pytest.skip("BPE merges file not available")


@pytest.fixture(scope="module")
def tok():
    return T.SimpleTokenizer(bpe_path=_bpe())


TEXTS = [str(t) for t in G["texts"]]


def test_vocab(tok):
    assert tok.vocab_size == int(G["vocab_size"][0]) == 49408
    assert (tok.sot_token_id, tok.eot_token_id) == (49406, 49407)


@pytest.mark.parametrize("clean", ["lower", "whitespace", "canonicalize"])
def test_ids_match_reference(clean):
    t = T.SimpleTokenizer(bpe_path=_bpe(), clean=clean)
    ids = t(TEXTS).numpy()
    ref = G[f"ids_{clean}"]
    bad = [i for i in range(len(TEXTS)) if not np.array_equal(ids[i], ref[i])]
    assert not bad, [(TEXTS[i], ids[i][:20].tolist(), ref[i][:20].tolist()) for i in bad[:3]]


def test_truncation_context16(tok):
    ids = tok(TEXTS, context_length=16).numpy()
    assert np.array_equal(ids, G["ids_ctx16"])
    long_row = ids[[i for i, t in enumerate(TEXTS) if t.startswith("a very long")][0]]
    assert long_row[-1] == tok.eot_token_id


def test_encode_decode(tok):
    off = 0
    for i, t in enumerate(TEXTS):
        n = int(G["enc_len"][i])
        ref = G["enc_flat"][off:off + n].tolist()
        off += n
        enc = tok.encode(t)
        assert enc == ref, t
        assert tok.decode(enc) == str(G["decoded"][i]), t


def test_additional_special_tokens():
    t = T.SimpleTokenizer(bpe_path=_bpe(), additional_special_tokens=["<extra_a>", "<extra_b>"])
    assert t.vocab_size == int(G["vocab_size"][1])
    assert np.array_equal(t(["x <extra_a> y <extra_b>", "plain"]).numpy(), G["ids_extra"])


def test_call_surface(tok):
    out = tok("a photo of a cat")                    # a single string -> [1, 77] int64
    assert out.shape == (1, 77) and out.dtype == torch.long
    assert tok([]).shape == (0, 77)
    os.environ.setdefault("CLIPEMBED_BPE_PATH", _bpe())
    assert torch.equal(T.tokenize(["a photo of a cat"]), out)
    assert T.get_tokenizer("ViT-B-16").context_length == 77


def test_prepare_data_text_half(monkeypatch):
    """prepare_data / prepare_data_clip .preprocess_text (data/utils.py:54-55, 69-70) tokenize with
    the ViT-L-14-336 tokenizer: same ids as the golden default-mode rows."""
    import clipembed
    monkeypatch.setenv("CLIPEMBED_BPE_PATH", _bpe())
    calls = []

    def proc(img):                     # a host-side image processor, applied per image and stacked
        calls.append(img)
        return torch.full((3, 4, 4), float(img))

    pd = clipembed.prepare_data_clip(proc)
    x = pd.preprocess_image([1, 2, 3])
    assert x.shape == (3, 3, 4, 4) and calls == [1, 2, 3]
    assert float(pd.preprocess_image(5)[0, 0, 0]) == 5.0
    ids = pd.preprocess_text(TEXTS[:4])
    ref = T.SimpleTokenizer(bpe_path=_bpe())(TEXTS[:4])
    assert ids.dtype == torch.long and torch.equal(ids, ref)
