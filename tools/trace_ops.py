"""Op-level attribution of one GPT training step with torch.profiler: which
framework ops launch which kernels / memcpys (complements rocprofv3's
kernel-level view).

    python tools/trace_ops.py [--hidden 4096 --layers 2 --batch 8 --seq 1024]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=40)
    a = ap.parse_args()
    import torch
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    here = os.path.dirname(os.path.abspath(__file__))
    cfg = C.get_config(os.path.join(here, "..", "fleetx_amd/configs/nlp/gpt/pretrain_gpt_345M_single_card.yaml"),
                       overrides=["Model.hidden_size=%d" % a.hidden, "Model.num_layers=%d" % a.layers,
                                  "Model.num_attention_heads=%d" % a.heads, "Model.vocab_size=50304",
                                  "Global.local_batch_size=%d" % a.batch,
                                  "Global.micro_batch_size=%d" % a.batch,
                                  "Global.global_batch_size=None", "Engine.mix_precision.dtype=bfloat16",
                                  "Data.Train.dataset.max_seq_len=%d" % a.seq,
                                  "Data.Train.dataset.name=SyntheticGPTDataset"], nranks=1)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    eng = EagerEngine(configs=cfg, module=build_module(cfg), mode="train")
    dev = eng.device
    B, S = a.batch, a.seq

    def batch():
        t = torch.randint(0, 50304, (B, S + 1), device=dev)
        return [t[:, :-1].contiguous(), torch.arange(S, device=dev).expand(B, S), t[:, 1:].contiguous(),
                torch.ones(B, S, device=dev)]
    for _ in range(2):
        eng._fit_impl(batch())
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        eng._fit_impl(batch())
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total",
                                                           row_limit=a.rows, max_name_column_width=60))
    for e in prof.events():
        if e.name == "aten::copy_" and e.device_type.name == "CPU":
            par = e.cpu_parent.name if e.cpu_parent is not None else "-"
            gpar = e.cpu_parent.cpu_parent if e.cpu_parent is not None else None
            gp = gpar.name if gpar is not None else "-"
            print("COPY", e.input_shapes, "<-", par, "<-", gp)
    # which CPU ops issued device memcpys
    for e in prof.events():
        if "Memcpy" in e.name or "memcpy" in e.name.lower():
            p = e.cpu_parent
            chain = []
            while p is not None and len(chain) < 4:
                chain.append(p.name)
                p = p.cpu_parent
            print("MEMCPY", e.name, "<-", " <- ".join(chain))
            q = e.cpu_parent
            while q is not None:
                if q.stack:
                    print("   stack:", " | ".join(fr for fr in q.stack if "fleetx_amd" in fr or "tools" in fr))
                    break
                q = q.cpu_parent


if __name__ == "__main__":
    main()
