"""ViT pretraining throughput on one MI355X (BASELINE config 5: ViT-g/14 bf16,
the per-GPU share of the DP=8 run): images/s and MFU of the full training
step (forward, backward, global-norm clip, AdamW) through the engine, on
synthetic images and random-init weights.

    python tools/bench_vit.py [--config fleetx_amd/configs/vis/vit/ViT_g_patch14_224_synthetic_dp8.yaml]
        [--steps 10 --warmup 3] [--recompute | --no-recompute] [-o Key=value ...]

Model FLOPs per image = 3 x forward (no recompute term, as the GPT MFU):
forward per token and layer = 2 x (4 h^2 + 2 h m) for the QKV / out / MLP
GEMMs + 4 s h for the attention products, plus the patch embedding
(2 x 3 p^2 x h per patch) and the head.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))


def vit_flops_per_image(m):
    h = m.embed_dim
    L = len(m.blocks)
    mlp = m.blocks[0].mlp.fc1.weight.shape[0]
    s = m.pos_embed.shape[1]
    p = m.patch_embed.patch_size
    layer = 2 * (4 * h * h + 2 * h * mlp) * s + 4 * s * s * h
    embed = 2 * 3 * p * p * h * (s - 1)
    return 3.0 * (L * layer + embed)


def main():
    ap = argparse.ArgumentParser()
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--config", default=os.path.join(
        here, "fleetx_amd/configs/vis/vit/ViT_g_patch14_224_synthetic_dp8.yaml"))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-recompute", action="store_true")
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("-o", "--override", action="append", default=[])
    args = ap.parse_args()
    import torch
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.utils.hw import PEAK_DENSE_FLOPS

    ov = list(args.override)
    if args.no_recompute:
        ov.append("Model.use_recompute=False")
    if args.recompute:
        ov.append("Model.use_recompute=True")
    cfg = C.get_config(args.config, overrides=ov, nranks=1)
    lr = cfg.Optimizer.lr
    if lr.get("name") == "ViTLRScheduler":  # as tools/train.py: steps per epoch from the data
        lr.setdefault("step_each_epoch",
                      cfg.Data.Train.dataset.get("num_samples", 100000)
                      // cfg.Data.Train.sampler.batch_size)
        lr.setdefault("epochs", cfg.Engine.get("num_train_epochs", 1))
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    module = build_module(cfg)
    eng = EagerEngine(configs=cfg, module=module, mode="train")
    B = cfg.Data.Train.sampler.batch_size
    size = cfg.Data.Train.dataset.get("image_size", 224)
    ncls = cfg.Data.Train.dataset.get("class_num", 1000)
    dev = eng.device
    g = torch.Generator(device=dev)
    g.manual_seed(1234)

    def batch():
        return [torch.randn(B, 3, size, size, device=dev, generator=g),
                torch.randint(0, ncls, (B,), device=dev, generator=g)]

    for _ in range(args.warmup):
        loss = eng._fit_impl(batch())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = eng._fit_impl(batch())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    net = module.model
    fpi = vit_flops_per_image(net)
    ips = B * args.steps / el
    dt = eng._dtype
    peak = PEAK_DENSE_FLOPS["bfloat16" if dt == torch.bfloat16 else "float16"]
    print(json.dumps({
        "metric": "images/sec ViT pretraining (1 GPU)", "model": cfg.Model.model.name,
        "value": round(ips, 1), "unit": "images/s", "ms_per_step": round(1000 * el / args.steps, 2),
        "batch": B, "steps": args.steps, "warmup": args.warmup,
        "dtype": str(dt).replace("torch.", ""), "recompute": bool(cfg.Model.use_recompute),
        "gflops_per_image": round(fpi / 1e9, 1), "mfu": round(ips * fpi / peak, 4),
        "final_loss": round(float(loss), 4), "data": "synthetic images, random-init weights",
        "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}), flush=True)


if __name__ == "__main__":
    main()
