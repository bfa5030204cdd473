"""Throughput benchmark of the CLIP ViT-L/14-336 embedding path (BASELINE.json configs[1]):
encode_image + encode_text of a synthetic batch (336x336 images, 77-token captions) per GPU,
L2-normalised, then (N > 1) an RCCL all-gather of both embedding sets and the local contrastive
logits [B, N*B] in both directions — the data-parallel step of loss.py:137-164 with local_loss.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Prints ONE JSON line (rank 0).  value = image-text pairs/s over all ranks (weak scaling: B pairs
per GPU per step), inputs resident in HBM before the timed region.  `roofline` reports the
dominant kernel (by total time in an untimed profile pass) measured with HIP events on its stream
over the timed steps (only its launches carry events there);
`cpu_baseline` times the f32 CPU oracle (oracle/clip_oracle.py, a restatement of the reference's
PyTorch CPU forward) on a bounded sample on this host.
"""
import argparse
import json
import os
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


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sd, cfg, n_pairs):
    """Time the f32 CPU oracle (the reference's algorithm restated in NumPy) on n_pairs pairs."""
    from oracle import clip_oracle as O
    from clipembed import weights as W
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = os.cpu_count() or 1
    imgs = W.synthetic_images(n_pairs, seed=5000)
    caps = W.synthetic_captions(n_pairs, seed=6000)
    O.encode_text(sd, caps[:1], cfg)          # warm-up (BLAS init)
    t0 = time.perf_counter()
    fi = O.encode_image(sd, imgs, cfg, normalize=True)
    ft = O.encode_text(sd, caps, cfg, normalize=True)
    O.get_logits(fi, ft, 100.0)
    dt = time.perf_counter() - t0
    return {"value": round(n_pairs / dt, 4), "unit": "pairs/s", "cores": int(threads), "kind": "port",
            "sample": f"{n_pairs} image-text pairs, full-depth ViT-L/14-336 f32 NumPy oracle "
                      f"(encode_image + encode_text + logits), {dt:.1f} s"}


def load_traffic(tag):
    """HBM bytes per launch of `tag` from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(tag, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="image-text pairs per GPU per step")
    ap.add_argument("--cpu-pairs", type=int, default=8, help="pairs in the bounded CPU-baseline sample (~10 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="do not bracket kernels with HIP events")
    ap.add_argument("--text-stream", action="store_true", help="run the text tower on a second stream")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import clipembed
    from clipembed import weights as W
    from clipembed.loss import all_gather_cat

    cfg = clipembed.get_model_config("ViT-L-14-336")
    t0 = time.time()
    sd = W.synthetic_state_dict(cfg)
    model = clipembed.CLIP(cfg)
    model.load_state_dict(sd)
    model.to(dev)
    B = args.batch
    model.engine.h  # noqa: B018
    from clipembed import _lib
    _lib.call("ce_reserve", model.engine.h, B, B)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000 + rank)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(B, seed=2000 + rank)).to(dev)
    scale = float(model.logit_scale.detach().exp())
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s, batch {B}/GPU, world {world}")

    side = torch.cuda.Stream(dev)
    main_stream = torch.cuda.current_stream(dev)

    def step():
        if args.text_stream:
            # the text tower (its own workspace in the engine) on a second stream, overlapping the
            # vision tower's tile tails and row kernels
            side.wait_stream(main_stream)
            with torch.cuda.stream(side):
                ft = model.encode_text(caps, normalize=True)
            fi = model.encode_image(imgs, normalize=True)
            main_stream.wait_stream(side)
            ft.record_stream(main_stream)
        else:
            fi = model.encode_image(imgs, normalize=True)
            ft = model.encode_text(caps, normalize=True)
        if world > 1:
            ai = all_gather_cat(fi, world)          # RCCL all-gather over xGMI
            at = all_gather_cat(ft, world)
            li, _ = model.logits(fi, at, scale, with_text_logits=False)
            lt, _ = model.logits(ft, ai, scale, with_text_logits=False)
        else:
            li, lt = model.logits(fi, ft, scale)
        return li, lt

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    timing = not args.no_timing
    profile = []
    if timing:
        # untimed profile pass: every kernel bracketed by HIP events -> per-kernel table (stderr) and
        # the dominant kernel; inside the timed region only that kernel's launches carry events
        model.engine.set_timing(True)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        profile = model.engine.kernel_stats()
        model.engine.set_timing(False)
        profile.sort(key=lambda s: -s["ms"])
        model.engine.set_timing(True, only=profile[0]["name"])
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
    stats = model.engine.kernel_stats() if timing else []
    if timing:
        model.engine.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    pairs = world * B * args.steps
    value = pairs / elapsed
    roof = None
    if stats:
        stats.sort(key=lambda s: -s["ms"])
        total_ms = sum(s["ms"] for s in profile)
        log("  per-kernel (profile pass, 2 steps, every launch bracketed by HIP events):")
        for s in profile:
            per = s["ms"] / max(1, s["launches"])
            log(f"  {s['name']:<14} {s['ms'] / 2:9.3f} ms/step  {100 * s['ms'] / total_ms:5.1f}%  "
                f"{s['launches'] // 2:4d} launches/step  "
                f"{(s['flops'] / s['launches']) / (per * 1e-3) / 1e12 if s['flops'] else 0:8.1f} TFLOP/s  "
                f"{(s['bytes'] / s['launches']) / (per * 1e-3) / 1e9:8.1f} GB/s")
        top = stats[0]
        per_ms = top["ms"] / top["launches"]
        if top["flops"] > 0:
            ach = (top["flops"] / top["launches"]) / (per_ms * 1e-3) / 1e12
            log(f"  timed region: {top['name']} {top['launches']} launches, avg {per_ms:.4f} ms")
            roof = {"bound": "mfma", "kernel": top["name"], "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                    "traffic": load_traffic(top["name"]), "avg_launch_ms": round(per_ms, 4),
                    "flops_per_launch": top["flops"] / top["launches"]}
        else:
            ach = (top["bytes"] / top["launches"]) / (per_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "kernel": top["name"], "achieved": round(ach, 2), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": load_traffic(top["name"])}
        roof["step_mfma_frac"] = round(value * FLOPS_PER_PAIR / 1e12 / world / PEAK_BF16_TFLOPS, 4)

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(sd, cfg, args.cpu_pairs)
        cpu["vs_gpu"] = round(value / cpu["value"], 1)

    out = {
        "metric": "image-text pairs/sec ViT-L/14-336",
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
        "config": {"workload": "CLIP ViT-L/14-336 encode_image + encode_text + normalise + contrastive logits "
                               "(BASELINE configs[1]: batch 256/GPU bf16)",
                   "batch_per_gpu": B, "global_batch": world * B, "image_size": 336, "context_length": 77,
                   "parallelism": f"dp{world}",
                   "exchange": "RCCL all_gather of L2-normalised embeddings" if world > 1 else "none"},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
