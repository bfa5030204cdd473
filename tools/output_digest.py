"""Bitwise digest of the engine's default-path outputs (A/B of two library builds: same inputs, same
weights, SHA-256 of every output array).  Used to show that a change which only removes or
restructures non-default code leaves the default outputs bit for bit unchanged.

    python tools/output_digest.py --out gpurun_out/digest_new.json
    CLIPEMBED_LIB=tools/ablib/libclipembed_r05.so python tools/output_digest.py --out gpurun_out/digest_old.json
    python tools/output_digest.py --compare gpurun_out/digest_old.json gpurun_out/digest_new.json

Workloads: the bench batch (B = 256 pooled image + text, pruned and every row, logits), token outputs
(B = 8), the unfolded f32-stream towers (B = 8), PACL ones / rope-after (B = 64), SPARC forward + loss
(B = 16) and one SPARC head training step (dropout on), and one NegCLIP training step (64 images + 96 captions: loss, flat gradient, first update).
"""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "clip-embeds_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def digest(t):
    import torch
    a = t.detach().contiguous()
    if a.dtype == torch.bfloat16:
        a = a.view(torch.int16)
    b = a.cpu().numpy().tobytes()
    return {"sha256": hashlib.sha256(b).hexdigest(), "shape": list(t.shape), "first": float(t.reshape(-1)[0])}


def run(out_path):
    import torch
    import clipembed
    from clipembed import weights as W
    from clipembed.pacl import SparcLoss, open_clip_pacl, open_clip_pacl_rope_after, sparc

    dev = torch.device("cuda", 0)
    cfg = clipembed.get_model_config("ViT-L-14-336")
    sd = W.synthetic_state_dict(cfg)
    res = {}
    m = clipembed.CLIP(cfg)
    m.load_state_dict(sd)
    m.to(dev)
    imgs = torch.from_numpy(W.synthetic_images(256, seed=1000)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(256, seed=2000)).to(dev)
    fi = m.encode_image(imgs, normalize=True)
    ft = m.encode_text(caps, normalize=True)
    il, tl = m.logits(fi, ft, 100.0)
    res.update(clip256_img=digest(fi), clip256_txt=digest(ft), clip256_logits=digest(il))
    m.engine.set_pooled_prune(False)
    res.update(clip256_img_every_row=digest(m.encode_image(imgs, normalize=True)),
               clip256_txt_every_row=digest(m.encode_text(caps, normalize=True)))
    m.engine.set_pooled_prune(True)
    m.visual.output_tokens = True
    m.output_text_tokens = True
    pi, ti = m.encode_image(imgs[:8])
    pt, tt = m.encode_text(caps[:8])
    res.update(tok_img_pooled=digest(pi), tok_img_tokens=digest(ti), tok_txt_pooled=digest(pt),
               tok_txt_tokens=digest(tt))
    m.visual.output_tokens = False
    m.output_text_tokens = False
    m.engine.set_ln_fold(False)
    res.update(unfolded_img=digest(m.encode_image(imgs[:8])), unfolded_txt=digest(m.encode_text(caps[:8])))
    m.engine.set_ln_fold(True)
    torch.cuda.synchronize()
    del m

    for name, cls in (("pacl", open_clip_pacl), ("pacl_rope_after", open_clip_pacl_rope_after)):
        mod = cls(cfg=cfg, clip_state_dict=sd)
        mod.init_synthetic_heads()
        mod.to(dev)
        oi, ot = mod(imgs[:64], caps[:64])
        res[f"{name}_img"] = digest(oi)
        res[f"{name}_txt"] = digest(ot)
        del mod
    sp = sparc(sigma=1.0 / 576, cfg=cfg, clip_state_dict=sd)
    sp.init_synthetic_heads()
    sp.to(dev)
    v, l, g, mask = sp(imgs[:16], caps[:16])
    loss = SparcLoss(0.1, engine=sp.engine)(v, l, g, mask)
    res.update(sparc_v=digest(v), sparc_l=digest(l), sparc_g=digest(g), sparc_loss=digest(loss.reshape(1)))
    # one SPARC head training step (round 6; builds without it skip these digests)
    if hasattr(clipembed, "SparcHeadTrainer"):
        st = clipembed.SparcHeadTrainer(sp, lr=1e-4, dropout=0.1, seed=5)
        sloss = st.compute_grads(imgs[:16], caps[:16])
        res.update(sparc_train_loss=digest(sloss.reshape(1)), sparc_train_grad=digest(st.grad))
        st.apply_update()
        res["sparc_train_param_after"] = digest(st.param)
        del st
    del sp
    torch.cuda.synchronize()

    m = clipembed.CLIP(cfg)
    m.load_state_dict(sd)
    m.to(dev)
    tr = clipembed.TextTowerTrainer(m, lr=5e-6, usehardtext=True)
    tcaps = torch.from_numpy(W.synthetic_captions(96, seed=2000)).to(dev)
    loss = tr.compute_grads(imgs[:64], tcaps)
    res.update(train_loss=digest(loss.reshape(1)), train_grad=digest(tr.grad))
    tr.apply_update()
    res["train_param_after"] = digest(tr.param)
    torch.cuda.synchronize()
    lib = os.environ.get("CLIPEMBED_LIB", "default")
    with open(out_path, "w") as f:
        json.dump({"lib": lib, "outputs": res}, f, indent=1)
    print(f"{len(res)} digests -> {out_path} ({lib})")


def compare(a_path, b_path):
    a = json.load(open(a_path))["outputs"]
    b = json.load(open(b_path))["outputs"]
    bad = [k for k in a if k not in b or a[k]["sha256"] != b[k]["sha256"]]
    for k in a:
        print(f"  {k:<24} {'equal' if k not in bad else 'DIFFERENT'}  {a[k]['first']:.6g} / "
              f"{b.get(k, {}).get('first', float('nan')):.6g}")
    print(f"{len(a) - len(bad)} of {len(a)} outputs bitwise equal")
    return 1 if bad else 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        sys.exit(compare(*args.compare))
    run(args.out)
