"""Weight loading: clipembed.load_checkpoint / load_state_dict mirror open_clip
factory.py:143-215 — .pt / {'state_dict'} wrapper / .safetensors, the 'module.' rule (strip only
when the FIRST key has it), logit_scale ndim fix, positional-embedding resize with the reference's
torch op — and the PACL checkpoint layout (module.clip_model.* + head keys, eval_pacl.py:380-388).
CPU only: the model keeps the host state dict until it is moved to a device."""
import math

import numpy as np
import pytest
import torch

import clipembed
from clipembed import weights as W
from clipembed.config import get_model_config


@pytest.fixture(scope="module")
def small_sd():
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    return cfg, {k: torch.from_numpy(np.asarray(v)) for k, v in W.synthetic_state_dict(cfg).items()}


def _same(model, sd):
    got = model.state_dict()
    for k, v in sd.items():
        if k == "logit_scale":
            assert float(got[k]) == pytest.approx(float(torch.as_tensor(v).reshape(())))
        else:
            assert torch.equal(torch.as_tensor(got[k]), torch.as_tensor(v)), k


@pytest.mark.parametrize("fmt", ["pt", "pt_wrapped", "pt_module", "safetensors"])
def test_checkpoint_formats_round_trip(tmp_path, small_sd, fmt):
    cfg, sd = small_sd
    sd = dict(sd)
    sd["logit_scale"] = torch.tensor([math.log(100.0)])          # 1-d, as some checkpoints store it
    path = tmp_path / ("w.safetensors" if fmt == "safetensors" else "w.pt")
    if fmt == "safetensors":
        from safetensors.torch import save_file
        save_file({k: v.contiguous() for k, v in sd.items()}, str(path))
    elif fmt == "pt":
        torch.save(sd, path)
    elif fmt == "pt_wrapped":
        torch.save({"state_dict": sd, "epoch": 3}, path)
    else:
        torch.save({"module." + k: v for k, v in sd.items()}, path)
    m = clipembed.CLIP(cfg)
    clipembed.load_checkpoint(m, str(path))
    _same(m, sd)
    assert m.logit_scale.ndim == 0 and float(m.logit_scale.detach()) == pytest.approx(math.log(100.0))
    direct = clipembed.CLIP(cfg)
    direct.load_state_dict({k: (v.reshape(()) if k == "logit_scale" else v) for k, v in sd.items()})
    for k, v in direct.state_dict().items():
        assert torch.equal(torch.as_tensor(m.state_dict()[k]), torch.as_tensor(v)), k


def test_module_prefix_rule_follows_first_key(tmp_path, small_sd):
    """factory.py:165-166 strips 'module.' from every key only when the FIRST key starts with it."""
    cfg, sd = small_sd
    keys = list(sd)
    mixed = {keys[0]: sd[keys[0]], "module." + keys[1]: sd[keys[1]]}
    path = tmp_path / "mixed.pt"
    torch.save(mixed, path)
    got = clipembed.load_state_dict(str(path))
    assert list(got) == [keys[0], "module." + keys[1]]
    first = {"module." + keys[0]: sd[keys[0]], "moduleX" + keys[1][1:]: sd[keys[1]]}
    torch.save(first, path)
    got = clipembed.load_state_dict(str(path))
    assert list(got) == [keys[0], keys[1][1:]]          # 'moduleX' + rest loses its first 7 characters


def test_pos_embed_resize_matches_reference_op(tmp_path, small_sd):
    """A 16 x 16 grid checkpoint into the 24 x 24 model: bicubic + antialias F.interpolate of the
    patch rows, class row kept (model.py:748-779)."""
    cfg, sd = small_sd
    sd = dict(sd)
    rng = np.random.default_rng(0)
    old = torch.from_numpy(rng.standard_normal((1 + 16 * 16, cfg.vision.width)).astype(np.float32))
    sd["visual.positional_embedding"] = old
    path = tmp_path / "grid16.pt"
    torch.save(sd, path)
    m = clipembed.CLIP(cfg)
    clipembed.load_checkpoint(m, str(path))
    got = torch.as_tensor(m.state_dict()["visual.positional_embedding"])
    assert tuple(got.shape) == (1 + 24 * 24, cfg.vision.width)
    img = old[1:].reshape(1, 16, 16, -1).permute(0, 3, 1, 2)
    ref = torch.nn.functional.interpolate(img, size=(24, 24), mode="bicubic", antialias=True, align_corners=False)
    ref = torch.cat([old[:1], ref.permute(0, 2, 3, 1).reshape(24 * 24, -1)])
    assert torch.equal(got, ref)


def test_pacl_checkpoint_layout(small_sd):
    """eval_pacl.py:380-388: PACL checkpoints hold module.clip_model.<open_clip name> + head keys."""
    from clipembed.pacl import open_clip_pacl
    cfg, sd = small_sd
    heads = {k: torch.from_numpy(np.asarray(v)) for k, v in W.synthetic_pacl_heads(cfg.with_pacl(768)).items()}
    ckpt = {"module.clip_model." + k: v for k, v in sd.items()}
    ckpt.update({"module." + k: v for k, v in heads.items()})
    mod = open_clip_pacl(cfg=cfg)
    mod.load_state_dict(ckpt)
    _same(mod.clip_model, sd)
    assert set(mod._heads) == set(heads) and all(torch.equal(mod._heads[k], heads[k]) for k in heads)


def test_pretrained_tag_needs_local_dir(monkeypatch):
    """eval_clip.py:21 passes pretrained='openai': the tag (pretrained.py:308-313) resolves to a
    local copy under $CLIPEMBED_PRETRAINED_DIR; unset, the error names the variable."""
    from clipembed.model import PRETRAINED_DIR_ENV, resolve_pretrained
    monkeypatch.delenv(PRETRAINED_DIR_ENV, raising=False)
    with pytest.raises(RuntimeError, match=PRETRAINED_DIR_ENV):
        clipembed.create_model("ViT-L-14-336", pretrained="openai")
    with pytest.raises(RuntimeError, match="not a known tag or valid file path"):
        resolve_pretrained("ViT-L-14-336", "laion2b_nonexistent")


@pytest.mark.parametrize("layout", ["vit_large_patch14_clip_336.openai/open_clip_model.safetensors",
                                    "vit_large_patch14_clip_336.openai/open_clip_pytorch_model.bin",
                                    "ViT-L-14-336/openai/open_clip_model.safetensors",
                                    "ViT-L-14-336-openai.safetensors"])
def test_pretrained_tag_resolves_local_copy(tmp_path, monkeypatch, layout):
    """create_model('ViT-L-14-336', pretrained='openai') loads the local copy through
    load_checkpoint (factory.py:390-404 + 171-215); the tag's quick_gelu=True against the GELU
    config warns as factory.py:435-445 does."""
    from clipembed.model import PRETRAINED_DIR_ENV, resolve_pretrained
    path = tmp_path / layout
    path.parent.mkdir(parents=True, exist_ok=True)
    sd = {"logit_scale": torch.tensor([math.log(100.0)]), "ln_final.weight": torch.arange(768, dtype=torch.float32)}
    if layout.endswith(".safetensors"):
        from safetensors.torch import save_file
        save_file(sd, str(path))
    else:
        torch.save(sd, path)
    monkeypatch.setenv(PRETRAINED_DIR_ENV, str(tmp_path))
    assert resolve_pretrained("ViT-L-14-336", "openai", quick_gelu=True) == str(path)
    with pytest.warns(UserWarning, match="QuickGELU mismatch"):
        m = clipembed.create_model("ViT-L-14-336", pretrained="openai")
    assert float(m.logit_scale.detach()) == pytest.approx(math.log(100.0))
    assert torch.equal(m.state_dict()["ln_final.weight"], sd["ln_final.weight"])
    (tmp_path / "empty").mkdir()
    monkeypatch.setenv(PRETRAINED_DIR_ENV, str(tmp_path / "empty"))
    with pytest.raises(RuntimeError, match="no checkpoint under"):
        resolve_pretrained("ViT-L-14-336", "openai")
