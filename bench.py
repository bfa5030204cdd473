"""Throughput benchmark of the CLIP ViT-L/14-336 embedding path, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload clip|pacl|negclip|sparc] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N > 1` without a launcher re-launches this script under torch.distributed.run as a child
process (before any GPU call) and exits with its status; it never silently runs one rank.

Workloads (BASELINE.json configs; a "step" is one pass of the hot path over one synthetic batch):
  clip     (default, configs[1], the headline metric) encode_image + encode_text of B = 256 pairs per
           GPU, L2-normalised; N > 1: RCCL all-gather of both embedding sets and the local
           contrastive logits [B, N*B] both ways (loss.py:137-164, local_loss).
  pacl     (configs[2]) PACL forward of B = 512 pairs per GPU (open_clip_pacl.forward, pacl.py:135-145:
           text tower + head, vision tower + patch head, fused patch alignment/pooling) + the PACL
           ClipLoss(0.1) (pacl.py:489-514; N > 1: RCCL all-gather of the pooled features, each rank's
           rows of the global logits, all-reduce of the CE sums: the value over the whole global batch,
           as train_pacl.py:34-36 computes it after nn.DataParallel's gather).
  negclip  (configs[3]) NegCLIP training step, locked image tower: 1024 pairs + 512 hard-negative
           captions per GPU, text tower backward, RCCL all-reduce of text gradients, AdamW.
  sparc    (configs[4]) the train_sparc.py step with precomputed text-token embeddings [B,77,768] +
           mask: frozen image tower, patch head in train mode (Dropout 0.1), patch x token similarity /
           alignment (pacl.py:455-478), SparcLoss, head backward and Adam (--sparc-forward: forward + loss
           value only); SparcLoss
           (pacl.py:516-584, temperature 0.1 as train_sparc.py:105; N > 1: RCCL all-gather of the
           [B,768] normalised patch / token means for the global term, the per-sample local term's sums
           and the global CE sums all-reduced: the loss over the whole global batch, as
           train_sparc.py:93,105 computes it after nn.DataParallel's gather) for B = 256 per GPU.

Prints ONE JSON line (rank 0).  value = image-text pairs/s over all ranks (weak scaling: B pairs
per GPU per step), inputs resident in HBM before the timed region.  `roofline` reports the
dominant kernel (by total time in an untimed profile pass), measured with HIP events on its stream
over the timed steps (only its launches carry events there); for pacl it also carries the pooling
kernel's HBM rate.  `cpu_baseline` times the reference's CPU forward (oracle/clip_torch_cpu.py: the
reference's own ATen calls, f32) on this host at batch 8, median of 3, at the host's core share
and at 8 threads.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "clip-embeds_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0          # HBM3E spec
FLOPS_PER_PAIR = 395.22e9      # open_clip/docs/model_profile.csv:65 (381.92 image + 13.30 text GFLOP)
IMAGE_FLOPS = 381.92e9
TEXT_FLOPS = 13.30e9
PACL_HEAD_FLOPS = 2.49e9       # PACL patch head per image (+ the pooling, counted below)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(nproc):
    """Run this script under torch.distributed.run with nproc ranks (a child process; no exec)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    log("launching:", " ".join(cmd))
    return subprocess.call(cmd)


# ----------------------------------------------------------------------------------- CPU baseline
def host_cores():
    for k in ("OMP_NUM_THREADS",):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(sd, cfg, batch=8, reps=3, warmup=3):
    """The reference's f32 CPU forward (encode_image + encode_text + logits) at `batch` pairs, `warmup`
    untimed iterations then the median of `reps`, at the host core share and at 8 threads (SURVEY
    §8(d))."""
    from oracle.clip_torch_cpu import TorchCLIP
    from clipembed import weights as W
    m = TorchCLIP(sd, cfg)
    imgs = torch.from_numpy(W.synthetic_images(batch, seed=5000))
    caps = torch.from_numpy(W.synthetic_captions(batch, seed=6000))
    prev = torch.get_num_threads()
    res = {}
    cores = host_cores()
    for n in sorted({cores, 8}, reverse=True):
        torch.set_num_threads(n)
        ts = []
        for it in range(warmup + reps):
            t0 = time.perf_counter()
            fi = m.encode_image(imgs, normalize=True)
            ft = m.encode_text(caps, normalize=True)
            m.get_logits(fi, ft, 100.0)
            if it >= warmup:
                ts.append(time.perf_counter() - t0)
        res[n] = float(np.median(ts))
    torch.set_num_threads(prev)
    out = {"value": round(batch / res[cores], 4), "unit": "pairs/s", "cores": cores, "kind": "port",
           "sample": f"{batch} image-text pairs per run, {warmup} warm-up runs, median of {reps}: full-depth "
                     f"ViT-L/14-336 f32 torch CPU forward with the reference's ATen calls (oracle/clip_torch_cpu.py), encode_image + "
                     f"encode_text + logits; {res[cores]:.2f} s at {cores} threads"}
    if 8 in res:
        out["value_8_threads"] = round(batch / res[8], 4)
    return out


def load_traffic(tag):
    """HBM bytes per launch of `tag` from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(tag, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def load_mfma_busy(tag):
    """Counter-based MFMA utilisation of `tag` (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE, one rocprofv3
    --pmc pass over this bench; tools/summarize_mfma.py -> profiles/<round>/mfma_busy.json, the latest
    round that has one), if measured."""
    for rnd in ("r06", "r05", "r04"):
        path = os.path.join(REPO, "profiles", rnd, "mfma_busy.json")
        try:
            with open(path) as f:
                d = json.load(f)["kernels"].get(tag)
        except (OSError, ValueError, KeyError):
            continue
        if not d:
            continue
        return {"mfma_busy": d["mfma_busy"], "clock_GHz": d["clock_GHz"], "frac_at_nominal": d["frac_at_nominal"],
                "source": f"profiles/{rnd}/mfma_busy.json"}
    return None


# ----------------------------------------------------------------------------------- workloads
def pooled_prune_flops(cfg, on=True, eot=None):
    """FLOPs per pair NOT executed by pooled-only calls (ce_set_pooled_prune): the image tower's last
    block runs out-proj, c_fc, c_proj and attention for the CLS row only; the text tower runs on the
    rows 0..EOT of each caption (packed; no later row reaches the EOT row under the causal mask) and
    its last block for the EOT row only.  Counted as the reference's profile counts a forward (full
    L x L attention; TEXT_FLOPS scaled by this model of the text work).  eot: EOT positions of the
    captions (None: text not pruned).  Returns (image, text) per pair."""
    if not on:
        return 0.0, 0.0
    v, t = cfg.vision, cfg.text
    Lv = (v.image_size // v.patch_size) ** 2 + 1
    img = (Lv - 1) * (2.0 * v.width ** 2 + 4.0 * v.width * v.mlp_width) + 4.0 * v.width * Lv * (Lv - 1)
    if eot is None:
        return img, 0.0
    L, D, F, nl = t.context_length, t.width, t.mlp_width, t.layers
    g = 2.0 * (4 * D * D + 2 * D * F)                        # GEMM FLOPs per row per block
    full = nl * (L * g + 4.0 * D * L * L)
    n = np.asarray(eot, np.float64) + 1.0
    run = (nl - 1) * (n * g + 4.0 * D * n * n) + (n * 6.0 * D * D + 4.0 * D * n + 2.0 * D * D + 4.0 * D * F)
    return img, TEXT_FLOPS * float(1.0 - run.mean() / full)


def build_clip(args, dev, rank, world):
    import clipembed
    from clipembed import _lib, weights as W
    from clipembed.loss import ClipLoss
    cfg = clipembed.get_model_config("ViT-L-14-336")
    sd = W.synthetic_state_dict(cfg)
    model = clipembed.CLIP(cfg)
    model.load_state_dict(sd)
    model.to(dev)
    B = args.batch or 256
    _lib.call("ce_reserve", model.engine.h, B, B)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000 + rank)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(B, seed=2000 + rank)).to(dev)
    scale = float(model.logit_scale.detach().exp())
    # the embedding exchange + local contrastive logits of open_clip's ClipLoss(local_loss=True)
    # (loss.py:137-164): N > 1 all-gathers both embedding sets over RCCL; N = 1 is one fused
    # logits launch both ways.  The same code runs on 2 gloo ranks in tests/test_dist_gloo.py.
    exch = ClipLoss(local_loss=True, rank=rank, world_size=world, engine=model.engine)

    # the two towers are independent until the logits: the text tower runs on a second HIP stream
    # so its kernels fill the image tower's partial last rounds and launch gaps (--serial-towers:
    # one stream)
    # --text-priority: the text tower's stream at high priority instead (its small kernels are
    # dispatched first whenever the image tower's persistent GEMMs free CUs)
    side = None if args.serial_towers else torch.cuda.Stream(dev, priority=-1 if args.text_priority else 0)
    # --tower-priority: the image tower (the critical path) on a high-priority stream, so the
    # dispatcher prefers its workgroups and the text tower only fills gaps
    hp = torch.cuda.Stream(dev, priority=-1) if (side is not None and args.tower_priority) else None

    def step(concurrent=True):
        if side is None or not concurrent:
            fi = model.encode_image(imgs, normalize=True)
            ft = model.encode_text(caps, normalize=True)
        else:
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                ft = model.encode_text(caps, normalize=True)
            if hp is None:
                fi = model.encode_image(imgs, normalize=True)
            else:
                hp.wait_stream(main)
                with torch.cuda.stream(hp):
                    fi = model.encode_image(imgs, normalize=True)
                main.wait_stream(hp)
                fi.record_stream(main)
            main.wait_stream(side)
            ft.record_stream(main)
        return exch.get_logits(fi, ft, scale)

    cfgd = {"workload": "CLIP ViT-L/14-336 encode_image + encode_text + normalise + contrastive logits "
                        "(BASELINE configs[1]: batch 256/GPU bf16)",
            "batch_per_gpu": B, "global_batch": world * B, "image_size": 336, "context_length": 77,
            "parallelism": f"dp{world}",
            "exchange": "RCCL all_gather of L2-normalised embeddings" if world > 1 else "none",
            "rows": ("every row" if args.no_pooled_prune else
                     "pooled-only calls: image last block for the CLS rows, text on rows 0..EOT (packed), "
                     "its last block for the EOT rows; outputs = the full computation's")}
    pi, pt = pooled_prune_flops(cfg, not args.no_pooled_prune, caps.cpu().numpy().argmax(1))
    return dict(engine=model.engine, step=step, pairs=B, flops_per_pair=FLOPS_PER_PAIR, sd=sd, cfg=cfg,
                flops_exec_per_pair=FLOPS_PER_PAIR - pi - pt,
                # profiles/pmc_traffic.json was measured on this default configuration
                pmc_tags=("gemm_fc_v", "gemm_qkv_v", "attn_v")
                if B == 256 and not args.no_pooled_prune else (),
                metric="image-text pairs/sec ViT-L/14-336", config=cfgd)


def build_pacl(args, dev, rank, world):
    import clipembed
    from clipembed import weights as W
    from clipembed.pacl import ClipLoss, open_clip_pacl, open_clip_pacl_rope_after
    cfg = clipembed.get_model_config("ViT-L-14-336")
    sd = W.synthetic_state_dict(cfg)
    cls = open_clip_pacl_rope_after if args.pacl_mode == "sigmoid_rope_after" else open_clip_pacl
    mod = cls(cfg=cfg, clip_state_dict=sd)
    mod.init_synthetic_heads()
    mod.to(dev)
    B = args.batch or 512
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000 + rank)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(B, seed=2000 + rank)).to(dev)
    # train_pacl.py:106: temperature 0.1; N > 1: the global-batch value from sharded rows (all-gather of
    # the features + all-reduce of 5 floats; tests/test_dist_gloo.py, tests/test_gpu_dist_loss.py)
    loss = ClipLoss(0.1, engine=mod.engine, rank=rank, world_size=world)
    pool_flops = 2.0 * 576 * 768 * (2 if cls.weight_mode else 1)

    if args.pacl_train:
        # the train_pacl.py:16-40 step with open_clip_pacl's heads: forward (dropout 0.1), ClipLoss, head
        # backward, Adam(lr 1e-4) (train_pacl.py:106-107)
        if cls is not open_clip_pacl:
            raise SystemExit("--pacl-train: the ones-weighted open_clip_pacl heads only")
        tr = clipembed.PaclHeadTrainer(mod, lr=1e-4, dropout=0.1, temperature=0.1, rank=rank, world_size=world)

        def step():
            out = tr.compute_grads(imgs, caps)
            tr.apply_update()
            return out
        cfgd = {"workload": "PACL head training step (open_clip_pacl, train_pacl.py): frozen towers, heads in train "
                            "mode, ClipLoss(0.1), head backward, Adam",
                "batch_per_gpu": B, "global_batch": world * B, "parallelism": f"dp{world}",
                "exchange": ("RCCL all_gather of the normalised features + all_reduce of the loss sums and the "
                             "head gradients") if world > 1 else "none"}
        return dict(engine=mod.engine, step=step, pairs=B, sd=sd, cfg=cfg, prunable=False,
                    flops_per_pair=FLOPS_PER_PAIR + 2.5 * PACL_HEAD_FLOPS,
                    metric="PACL image-text pairs/sec ViT-L/14-336 (training)", config=cfgd)

    def step():
        oi, ot = mod(imgs, caps)
        return loss(oi, ot)

    cfgd = {"workload": f"PACL patch-token forward ({cls.__name__}) + patch alignment/pooling + PACL ClipLoss "
                        "(BASELINE configs[2]: batch 512/GPU bf16)",
            "batch_per_gpu": B, "global_batch": world * B, "image_size": 336, "context_length": 77,
            "parallelism": f"dp{world}", "pacl_mode": args.pacl_mode,
            "exchange": ("RCCL all_gather of the pooled features [B,768] x2 + all_reduce of the loss's CE sums "
                         "(global-batch ClipLoss value)") if world > 1 else "none"}
    _, pt = pooled_prune_flops(cfg, not args.no_pooled_prune, caps.cpu().numpy().argmax(1))  # pooled-only text
    return dict(engine=mod.engine, step=step, pairs=B, sd=sd, cfg=cfg,
                flops_per_pair=FLOPS_PER_PAIR + PACL_HEAD_FLOPS + pool_flops,
                flops_exec_per_pair=FLOPS_PER_PAIR + PACL_HEAD_FLOPS + pool_flops - pt,
                # profiles/pmc_traffic.json's pacl_pool entry was measured on this default configuration
                pmc_tags=("pacl_pool",) if B == 512 and args.pacl_mode == "ones" else (),
                metric="PACL image-text pairs/sec ViT-L/14-336", config=cfgd, hbm_kernel="pacl_pool")


def build_negclip(args, dev, rank, world):
    import clipembed
    from clipembed import weights as W
    cfg = clipembed.get_model_config("ViT-L-14-336")
    sd = W.synthetic_state_dict(cfg)
    m = clipembed.CLIP(cfg)
    m.load_state_dict(sd)
    m.to(dev)
    B = args.batch or 1024
    K = args.hard if args.hard is not None else B // 2
    tr = clipembed.TextTowerTrainer(m, lr=5e-6, usehardtext=K > 0, rank=rank, world_size=world)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000 + rank)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(B + K, seed=2000 + rank)).to(dev)

    def step():
        loss = tr.compute_grads(imgs, caps)
        tr.apply_update()
        return loss

    # image forward + text forward/backward (x3) over B + K captions
    flops = IMAGE_FLOPS + 3.0 * TEXT_FLOPS * (B + K) / B
    cfgd = {"workload": "open_clip NegCLIP training step, locked image tower, text tower AdamW "
                        "(BASELINE configs[3]: 1024 pairs + hard negatives per GPU, local loss, gather with grad)",
            "batch_per_gpu": B, "hard_negatives_per_gpu": K, "global_batch": world * B, "parallelism": f"dp{world}",
            "exchange": ("RCCL all_gather of embeddings + sizes, reduce_scatter of their gradients, "
                         "all_reduce of text gradients") if world > 1 else "none"}
    pi, _ = pooled_prune_flops(cfg, not args.no_pooled_prune)     # locked image tower: pooled-only
    return dict(engine=m.engine, step=step, pairs=B, flops_per_pair=flops, sd=sd, cfg=cfg,
                flops_exec_per_pair=flops - pi,
                metric="NegCLIP training image-text pairs/sec ViT-L/14-336", config=cfgd)


def build_sparc(args, dev, rank, world):
    import clipembed
    from clipembed import weights as W
    from clipembed.pacl import SparcLoss, sparc, sparc_rope
    cfg = clipembed.get_model_config("ViT-L-14-336")
    sd = W.synthetic_state_dict(cfg)
    cls = sparc_rope if args.sparc_rope else sparc
    mod = cls(sigma=1.0 / 576, cfg=cfg, clip_state_dict=sd)
    mod.init_synthetic_heads()
    mod.to(dev)
    B, T, P, D = args.batch or 256, 77, 576, 768
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000 + rank)).to(dev)
    # precomputed text-token embeddings (the train_sparc.py "LLM embeddings" input) + EOT mask
    g = torch.Generator(device="cpu").manual_seed(3000 + rank)
    l_tok = (torch.randn(B, T, D, generator=g) * 0.5).to(dev)
    eot = torch.randint(6, 42, (B,), generator=g)
    mask = (torch.arange(T).expand(B, -1) <= eot[:, None]).float().to(dev)
    sim_flops = 2.0 * T * P * D
    fwd_flops = IMAGE_FLOPS + PACL_HEAD_FLOPS + 2 * sim_flops + 2.0 * T * T * D
    if args.sparc_forward:
        loss_fn = SparcLoss(0.1, engine=mod.engine, rank=rank, world_size=world)     # train_sparc.py:105

        def step():
            v = mod.forward_visual(imgs)
            gr, ln = mod.align(v, l_tok)
            return loss_fn(v, ln, gr, mask)
        flops, what = fwd_flops, "forward + SparcLoss value"
    else:
        # the train_sparc.py:29-37 step: frozen image tower, heads in train mode (Dropout 0.1), SparcLoss,
        # backward through the alignment and the patch head, Adam(lr 1e-4) (train_sparc.py:91,106)
        tr = clipembed.SparcHeadTrainer(mod, lr=1e-4, dropout=0.1, temperature=0.1, rank=rank, world_size=world)

        def step():
            loss = tr.compute_grads(imgs, l_token_embed=l_tok, language_mask=mask)
            tr.apply_update()
            return loss
        # backward: weight gradients of the head (1x its forward; the hidden layer's input gradient adds
        # ~0.5x) and both operand gradients of the similarity / grouping products (2x)
        flops = fwd_flops + 1.5 * PACL_HEAD_FLOPS + 2 * (2 * sim_flops)
        what = "training step: forward (dropout 0.1) + SparcLoss + head backward + Adam"
    cfgd = {"workload": f"SPARC ({cls.__name__}) {what}: image tower + patch head, patch x token similarity / "
                        "alignment, SparcLoss with precomputed text-token embeddings (BASELINE configs[4]: batch 256/GPU)",
            "batch_per_gpu": B, "global_batch": world * B, "tokens": T, "patches": P, "dim": D,
            "parallelism": f"dp{world}", "loss_temperature": 0.1,
            "exchange": ("RCCL all_gather of the normalised patch / token means [B,768] x2 + all_reduce of the "
                         "5 loss partial sums" + ("" if args.sparc_forward else " + all_reduce of the head gradients")
                         ) if world > 1 else "none"}
    return dict(engine=mod.engine, step=step, pairs=B, sd=sd, cfg=cfg, flops_per_pair=flops, prunable=False,
                metric="SPARC image-text pairs/sec ViT-L/14-336" + ("" if args.sparc_forward else " (training)"),
                config=cfgd)


BUILDERS = {"clip": build_clip, "pacl": build_pacl, "negclip": build_negclip, "sparc": build_sparc}


def gloo_device_reduce_scatter():
    """Rehearsal backend only (--dist-backend gloo): some torch builds' gloo has no reduce_scatter for
    device tensors; the NegCLIP trainer's one reduce_scatter_tensor is then staged through host memory
    in this process.  The RCCL path (the default backend) never takes this."""
    try:
        o = torch.zeros(2, device="cuda")
        dist.reduce_scatter_tensor(o, torch.ones(2 * dist.get_world_size(), device="cuda"))
        return False
    except (RuntimeError, ValueError, NotImplementedError):
        real = dist.reduce_scatter_tensor

        def host_staged(output, input, op=dist.ReduceOp.SUM, group=None, async_op=False):
            o = output.cpu()
            real(o, input.cpu(), op=op, group=group)
            output.copy_(o)

        dist.reduce_scatter_tensor = host_staged
        log("gloo: reduce_scatter of device tensors staged through host memory (rehearsal backend)")
        return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(BUILDERS), default="clip")
    ap.add_argument("--batch", type=int, default=0, help="pairs per GPU per step (0 = the workload's config)")
    ap.add_argument("--hard", type=int, default=None, help="negclip: hard-negative captions per GPU (default B/2)")
    ap.add_argument("--pacl-mode", choices=["ones", "sigmoid_rope_after"], default="ones")
    ap.add_argument("--sparc-rope", action="store_true")
    ap.add_argument("--pacl-train", action="store_true",
                    help="pacl: time the train_pacl.py head training step instead of the forward")
    ap.add_argument("--sparc-forward", action="store_true",
                    help="sparc: time the forward + loss value only (default: the full training step)")
    ap.add_argument("--cpu-batch", type=int, default=8, help="pairs per CPU-baseline run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="do not bracket kernels with HIP events")
    ap.add_argument("--serial-towers", action="store_true", help="clip: both towers on one stream")
    ap.add_argument("--tower-priority", action="store_true", help="clip: image tower on a high-priority stream")
    ap.add_argument("--text-priority", action="store_true", help="clip: text tower on a high-priority stream")
    ap.add_argument("--attn-var", type=int, default=-1, help="attention forward variant for A/B (-1 = default)")
    ap.add_argument("--gemm-variant", type=int, default=-1, help="GEMM variant bits for A/B (-1 = default)")
    ap.add_argument("--no-pooled-prune", action="store_true",
                    help="run every tower's last block for all rows (A/B of ce_set_pooled_prune)")
    ap.add_argument("--no-every-row", action="store_true",
                    help="skip the second timed leg with the pooled prune off (`every_row` in the JSON line)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: torch.distributed backend (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank code path with every rank on one device, --share-device)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal of the N > 1 path on a one-GPU box; needs gloo: "
                         "RCCL runs one rank per device)")
    ap.add_argument("--gemm-stagger", type=int, default=-1,
                    help="first-round stagger of the persistent residual GEMMs (x s_sleep 127, odd slots; A/B)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"error: WORLD_SIZE={world} but --gpus={args.gpus}")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_device and args.dist_backend != "gloo":
        log("error: --share-device needs --dist-backend gloo (RCCL runs one rank per device)")
        sys.exit(2)
    dev_index = 0 if args.share_device else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            gloo_device_reduce_scatter()

    if args.attn_var >= 0:
        from clipembed import _lib
        _lib.lib().ce_set_attn_variant(args.attn_var)
    if args.gemm_variant >= 0:
        from clipembed import _lib
        _lib.lib().ce_set_gemm_variant(args.gemm_variant)
    if args.no_pooled_prune:
        os.environ["CE_POOLED_PRUNE"] = "0"          # read at ce_create
    if args.gemm_stagger >= 0:
        from clipembed import _lib
        L = _lib.lib()
        prev = L.ce_set_gemm_schedule(1)
        L.ce_set_gemm_schedule((prev & 0xffff) | ((args.gemm_stagger + 1) << 24))
    t0 = time.time()
    W = BUILDERS[args.workload](args, dev, rank, world)
    engine, step = W["engine"], W["step"]
    B = W["pairs"]
    log(f"[rank {rank}] {args.workload}: setup {time.time() - t0:.1f}s, batch {B}/GPU, world {world}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    timing = not args.no_timing
    profile = []
    if timing:
        # untimed profile pass: every kernel bracketed by HIP events -> per-kernel table (stderr) and
        # the dominant kernel; inside the timed region only that kernel's launches carry events
        engine.set_timing(True)
        for _ in range(2):
            step(concurrent=False) if args.workload == "clip" else step()
        torch.cuda.synchronize()
        profile = engine.kernel_stats()
        engine.set_timing(False)
        profile.sort(key=lambda s: -s["ms"])
        engine.set_timing(True, only=profile[0]["name"])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    stats = engine.kernel_stats() if timing else []
    if timing:
        engine.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # the same K steps with every row of the last blocks computed (pooled prune off):
    # reported beside `value` so the step is also measured without the dead-row skipping
    every_row = None
    if W.get("prunable", True) and not args.no_pooled_prune and not args.no_every_row:
        prev = engine.set_pooled_prune(False)
        step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el2 = time.perf_counter() - t1
        engine.set_pooled_prune(prev)
        if world > 1:
            t = torch.tensor([el2], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el2 = float(t.item())
        v2 = world * B * args.steps / el2
        every_row = {"value": round(v2, 2), "ms_per_step": round(1000 * el2 / args.steps, 3),
                     "model_flops_frac": round(v2 * W["flops_per_pair"] / 1e12 / world / PEAK_BF16_TFLOPS, 4)}

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    value = world * B * args.steps / elapsed
    roof = None
    if stats:
        stats.sort(key=lambda s: -s["ms"])
        total_ms = sum(s["ms"] for s in profile)
        log("  per-kernel (profile pass, 2 steps, every launch bracketed by HIP events):")
        for s in profile:
            per = s["ms"] / max(1, s["launches"])
            log(f"  {s['name']:<16} {s['ms'] / 2:9.3f} ms/step  {100 * s['ms'] / total_ms:5.1f}%  "
                f"{s['launches'] // 2:4d} launches/step  "
                f"{(s['flops'] / s['launches']) / (per * 1e-3) / 1e12 if s['flops'] else 0:8.1f} TFLOP/s  "
                f"{(s['bytes'] / s['launches']) / (per * 1e-3) / 1e9:8.1f} GB/s")
        top = stats[0]
        per_ms = top["ms"] / top["launches"]
        log(f"  timed region: {top['name']} {top['launches']} launches, avg {per_ms:.4f} ms")
        if top["flops"] > 0:
            ach = (top["flops"] / top["launches"]) / (per_ms * 1e-3) / 1e12
            roof = {"bound": "mfma", "kernel": top["name"], "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                    "traffic": load_traffic(top["name"]) if top["name"] in W.get("pmc_tags", ()) else None,
                    "avg_launch_ms": round(per_ms, 4),
                    "flops_per_launch": top["flops"] / top["launches"],
                    # the same kernel's MFMA-pipe busy fraction from hardware counters (committed profile)
                    "counters": load_mfma_busy(top["name"]) if args.workload == "clip" else None}
        else:
            ach = (top["bytes"] / top["launches"]) / (per_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "kernel": top["name"], "achieved": round(ach, 2), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
                    "traffic": load_traffic(top["name"]) if top["name"] in W.get("pmc_tags", ()) else None}
        # executed FLOPs (the pooled-only prune skips part of the last blocks) and the reference
        # model's FLOPs per pair (open_clip's profile), both over the dense bf16 peak
        fx = W.get("flops_exec_per_pair", W["flops_per_pair"])
        roof["step_mfma_frac"] = round(value * fx / 1e12 / world / PEAK_BF16_TFLOPS, 4)
        roof["model_flops_frac"] = round(value * W["flops_per_pair"] / 1e12 / world / PEAK_BF16_TFLOPS, 4)
        hk = W.get("hbm_kernel")
        if hk:
            hs = [s for s in profile if s["name"] == hk]
            if hs:
                s = hs[0]
                per = s["ms"] / s["launches"]
                gbs = (s["bytes"] / s["launches"]) / (per * 1e-3) / 1e9
                roof["hbm_kernel"] = {"kernel": hk, "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                      "frac": round(gbs / PEAK_HBM_GBS, 4), "avg_launch_ms": round(per, 4),
                                      "bytes_per_launch": s["bytes"] / s["launches"],
                                      "traffic": load_traffic(hk) if hk in W.get("pmc_tags", ()) else None}

    cpu = None
    if world == 1 and not args.no_cpu_baseline and args.workload == "clip":
        cpu = cpu_baseline(W["sd"], W["cfg"], args.cpu_batch)
        cpu["vs_gpu"] = round(value / cpu["value"], 1)

    if world > 1:
        W["config"]["dist_backend"] = args.dist_backend + (" (every rank on cuda:0: rehearsal, not a scaling number)"
                                                           if args.share_device else "")
    out = {
        "metric": W["metric"],
        "value": round(value, 2),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (deterministic uniform 336x336 images, 5-40 token captions; random-init weights)",
        "config": W["config"],
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if every_row:
        out["every_row"] = every_row
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
