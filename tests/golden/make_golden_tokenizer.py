"""Golden token ids from the REFERENCE tokenizer (open_clip tokenizer.py SimpleTokenizer), for the
C++ BPE (csrc/tokenizer.cpp) via clipembed.tokenizer.

Runs only in the build container: imports open_clip/src/open_clip/tokenizer.py from the read-only
reference tree with ftfy stubbed to the identity (ftfy is not installed) and writes
inputs (the texts) and outputs (ids, decoded strings) to tests/golden/tokenizer.npz.  No reference
source or data file is copied.

    python tests/golden/make_golden_tokenizer.py
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TOK_PY = "/root/reference/open_clip/src/open_clip/tokenizer.py"

TEXTS = [
    "a photo of a cat",
    "A dog to the LEFT of a tree!",
    "A mug on top of a table", "a mug under a table", "A bowl in front of a laptop",
    "Is the butterfly's wing visible?", "the cat's toy isn't here; we'll see, they've gone, I'm sure, you'd go, we're ok",
    "SHE'LL GO, IT'S, THEY'D", "rock'n'roll ''quoted'' 'single'",
    "1234 apples and 56.78 kg at 09:30", "   leading and   trailing   spaces\t\ttabs\nnewline  ",
    "", " ", "!!!???...", "hello,world;foo:bar(baz)[qux]{quux}",
    "café naïve résumé Ångström", "café decomposed e-acute", "北京的天安门广场", "Москва — столица России",
    "مرحبا بالعالم", "emoji 😀🐱👍🏽 mixed", "x² + y³ = z⁴, Ⅻ, ٣٤٥, ½", "ſtraße long s", "ﬁ ligature", "zero\u200bwidth nbsp\u00a0here\u3000ideographic\u2028sep",
    "&amp; &lt;b&gt; &quot;html&quot; &amp;amp; &#39;x&#39; &#x263A;",
    "<start_of_text> literal specials <end_of_text>", "<START_OF_TEXT> upper",
    "curly ’ apostrophe don’t", "under_score snake_case-dash/slash\\back",
    "a very long caption " + " ".join(f"word{i}" for i in range(120)),
    "supercalifragilisticexpialidocious antidisestablishmentarianism",
    "The photo shows two red apples and a green pear on a wooden table next to a window.",
]


def load_reference():
    ft = types.ModuleType("ftfy")
    ft.fix_text = lambda s: s
    sys.modules["ftfy"] = ft
    spec = importlib.util.spec_from_file_location("oc_tokenizer_reference", TOK_PY)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    mod = load_reference()
    out = {"texts": np.array(TEXTS)}
    for clean in ("lower", "whitespace", "canonicalize"):
        tok = mod.SimpleTokenizer(clean=clean)
        out[f"ids_{clean}"] = tok(TEXTS).numpy().astype(np.int64)
    tok = mod.SimpleTokenizer()
    out["ids_ctx16"] = tok(TEXTS, context_length=16).numpy().astype(np.int64)
    enc = [tok.encode(t) for t in TEXTS]
    out["enc_len"] = np.array([len(e) for e in enc], dtype=np.int64)
    out["enc_flat"] = np.array([i for e in enc for i in e], dtype=np.int64)
    out["decoded"] = np.array([tok.decode(e) for e in enc])
    extra = mod.SimpleTokenizer(additional_special_tokens=["<extra_a>", "<extra_b>"])
    out["ids_extra"] = extra(["x <extra_a> y <extra_b>", "plain"]).numpy().astype(np.int64)
    out["vocab_size"] = np.array([tok.vocab_size, extra.vocab_size], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "tokenizer.npz"), **out)
    print("wrote tokenizer.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
