"""Reference-checkpoint importer: a Paddle-layout ``.pdparams``
(pickled numpy dict, ``[in, out]`` Linear weights, reference names) written by
this test from a tiny model's weights loads into a fresh model and reproduces
its logits; code-executing pickles are refused."""
import os
import pickle

import numpy as np
import pytest
import torch

from fleetx_amd.utils import paddle_import as PI

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "fleetx_amd", "configs", "nlp", "gpt", "pretrain_gpt_345M_single_card.yaml")


def _module(seed):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    ov = ["Model.hidden_size=64", "Model.num_layers=2", "Model.num_attention_heads=4",
          "Model.vocab_size=256", "Model.max_position_embeddings=64", "Global.device=cpu",
          "Model.hidden_dropout_prob=0.0", "Model.attention_probs_dropout_prob=0.0",
          "Data.Train.dataset.name=SyntheticGPTDataset", "Global.seed=%d" % seed]
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    return build_module(cfg)


def _to_paddle_names(sd):
    """Inverse of the importer's map: what ``paddle.save`` of the reference model holds."""
    out = {}
    for k, v in sd.items():
        a = v.detach().float().numpy()
        if k == "gpt.embeddings.position_embeddings":
            out["gpt.embeddings.position_embeddings.weight"] = a
        elif k == "gpt.embeddings.word_embeddings.weight":
            out[k] = a
        elif k.startswith("gpt.final_ln."):
            out["gpt.decoder.norm." + k.split(".")[-1]] = a
        else:
            _, _, i, rest = k.split(".", 3)
            inv = {v2[0]: (k2, v2[1]) for k2, v2 in PI._SUB.items()}
            name, tr = inv[rest]
            out["gpt.decoder.layers.%s.%s" % (i, name)] = a.T.copy() if tr else a
    out["StructuredToParameterName@@"] = {k: "param_%d" % i for i, k in enumerate(out)}
    return out


def test_import_reproduces_logits(tmp_path):
    src = _module(1)
    path = tmp_path / "model.pdparams"
    with open(path, "wb") as f:
        pickle.dump(_to_paddle_names(src.model.state_dict()), f, protocol=2)
    dst = _module(2)
    with torch.no_grad():
        for prm in dst.model.parameters():
            prm.add_(0.05 * torch.randn_like(prm))
    ids = torch.randint(0, 256, (2, 16))
    pos = torch.arange(16).expand(2, 16)
    with torch.no_grad():
        before = dst.model(ids, pos)
        PI.load_into_model(dst.model, str(path))
        a, b = src.model(ids, pos), dst.model(ids, pos)
    a = a[0] if isinstance(a, tuple) else a
    b = b[0] if isinstance(b, tuple) else b
    before = before[0] if isinstance(before, tuple) else before
    assert not torch.allclose(a, before)
    assert torch.allclose(a, b, atol=1e-5)


def test_split_qkv_packing():
    h, heads = 8, 2
    q, k, v = (np.random.randn(h, h).astype(np.float32) for _ in range(3))
    sd = {"gpt.decoder.layers.0.self_attn.%s_proj.weight" % n: w for n, w in zip("qkv", (q, k, v))}
    fused = PI._pack_split_qkv(sd, heads)["gpt.decoder.layers.0.self_attn.qkv_proj.weight"]
    d = h // heads
    # per head: [q_h | k_h | v_h] (reference reshape [.., heads, 3*d] then split)
    f = fused.reshape(h, heads, 3, d)
    assert np.array_equal(f[:, 1, 0], q[:, d:2 * d]) and np.array_equal(f[:, 0, 2], v[:, :d])


def test_refuses_code_execution(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    data = pickle.dumps({"w": Evil()})
    with pytest.raises(pickle.UnpicklingError):
        PI.load_paddle_state(data)


def test_convert_cli(tmp_path):
    import subprocess
    import sys
    src = _module(1)
    path = tmp_path / "model.pdparams"
    with open(path, "wb") as f:
        pickle.dump(_to_paddle_names(src.model.state_dict()), f, protocol=4)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "convert_paddle_ckpt.py"),
                        "--src", str(path), "--dst", str(tmp_path / "out")],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout
    sd = torch.load(tmp_path / "out" / "model.pdparams", weights_only=True)
    ref = src.model.state_dict()
    assert set(sd) == set(ref)
    assert all(torch.allclose(sd[k], ref[k].float()) for k in ref)
