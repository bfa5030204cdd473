import sys, os
sys.path[:0] = [os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "clip-embeds_amd"), os.environ.get("GRAFT_REPO_ROOT", "/root/repo")]
import numpy as np, torch, clipembed
from clipembed import weights as W, _lib
from clipembed.config import get_model_config
from oracle import clip_oracle as O

def cd(a, b):
    a = np.asarray(a, np.float64).reshape(-1, a.shape[-1]); b = np.asarray(b, np.float64).reshape(-1, b.shape[-1])
    c = (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
    return float((1 - c).max())
cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
sd = W.synthetic_state_dict(cfg)
m = clipembed.CLIP(cfg); m.load_state_dict(sd); m.to("cuda")
caps = torch.from_numpy(W.synthetic_captions(8, seed=78))
m.output_text_tokens = True
_, otok = O.encode_text(sd, caps.numpy(), cfg, output_tokens=True)
res = {}
for name, fold, hl, auto in (("hl", 1, 1, 1), ("f32", 1, 0, 1), ("unfold", 0, 1, 1), ("hl_auto0", 1, 1, 0), ("f32_auto0", 1, 0, 0)):
    m._engine.set_ln_fold(bool(fold)); m._engine.set_resid_hl(bool(hl))
    pa = _lib.lib().ce_set_gemm_auto(auto); ps = _lib.lib().ce_set_gemm_splitk(auto)
    p, t = m.encode_text(caps); torch.cuda.synchronize()
    _lib.lib().ce_set_gemm_auto(pa); _lib.lib().ce_set_gemm_splitk(ps)
    res[name] = t.cpu().numpy()
    print(name, "vs oracle tokens", cd(res[name], otok), flush=True)
for a in res:
    for b in res:
        if a < b: print(a, b, cd(res[a], res[b]))
