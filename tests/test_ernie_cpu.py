"""ERNIE (reference C23/C33/K22): post-LN encoder layer vs torch's
TransformerEncoderLayer, padding-mask semantics, heads, dynamic MLM masking
and an end-to-end pretraining run through tools/train.py."""
import os

import numpy as np

import torch

from fleetx_amd.models.language_model.ernie import (ErnieModel, ErnieForPretraining,
                                                    ErnieForMaskedLM, ErnieForMultipleChoice,
                                                    ErniePretrainingCriterion, mlm_mask)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tiny(**kw):
    cfg = dict(vocab_size=96, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
               intermediate_size=64, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
               max_position_embeddings=64)
    cfg.update(kw)
    return ErnieModel(**cfg)


def test_encoder_layer_matches_torch_post_ln():
    torch.manual_seed(0)
    m = _tiny().eval()
    layer = m.encoder[0]
    with torch.no_grad():
        for p in layer.parameters():
            if p.ndim == 1:
                p.add_(0.1 * torch.randn_like(p))
    h, H = 32, 4
    d = h // H
    ref = torch.nn.TransformerEncoderLayer(h, H, 64, dropout=0.0, activation="gelu",
                                           layer_norm_eps=1e-12, batch_first=True,
                                           norm_first=False).eval()
    with torch.no_grad():
        w = layer.qkv.weight.view(H, 3, d, h).permute(1, 0, 2, 3).reshape(3 * h, h)
        bq = layer.qkv.bias.view(H, 3, d).permute(1, 0, 2).reshape(3 * h)
        ref.self_attn.in_proj_weight.copy_(w)
        ref.self_attn.in_proj_bias.copy_(bq)
        ref.self_attn.out_proj.weight.copy_(layer.out_proj.weight)
        ref.self_attn.out_proj.bias.copy_(layer.out_proj.bias)
        ref.linear1.weight.copy_(layer.linear1.weight)
        ref.linear1.bias.copy_(layer.linear1.bias)
        ref.linear2.weight.copy_(layer.linear2.weight)
        ref.linear2.bias.copy_(layer.linear2.bias)
        for a, b in ((ref.norm1, layer.norm1), (ref.norm2, layer.norm2)):
            a.weight.copy_(b.weight)
            a.bias.copy_(b.bias)
    x = torch.randn(3, 10, h)
    pad = torch.zeros(3, 10, dtype=torch.bool)
    pad[1, 7:] = True
    pad[2, 3:5] = True
    out = layer(x, pad.float() * -1e4)
    exp = ref(x, src_key_padding_mask=pad)
    assert torch.allclose(out, exp, atol=2e-5), (out - exp).abs().max()


def test_default_mask_is_pad_token_and_2d_mask():
    torch.manual_seed(1)
    m = _tiny().eval()
    ids = torch.randint(1, 96, (2, 12))
    ids[0, 9:] = 0
    seq, pooled = m(ids)
    assert seq.shape == (2, 12, 32) and pooled.shape == (2, 32)
    am = (ids != 0).long()
    seq2, _ = m(ids, attention_mask=am)
    assert torch.allclose(seq, seq2, atol=1e-6)
    # keys that are padding do not influence the other tokens
    ids2 = ids.clone()
    ids2[0, 9:] = 0
    ids2[0, 10] = 0
    seq3, _ = m(ids2)
    assert torch.allclose(seq[0, :9], seq3[0, :9], atol=1e-6)


def test_heads_and_criterion():
    torch.manual_seed(2)
    model = ErnieForPretraining(_tiny())
    ids = torch.randint(1, 96, (2, 8))
    pos = torch.tensor([1, 5, 9, 14])
    scores, rel = model(ids, masked_positions=pos)
    assert scores.shape == (4, 96) and rel.shape == (2, 2)
    # decoder tied to word embeddings
    assert model.cls.predictions.decoder_weight is model.ernie.embeddings.word_embeddings.weight
    labels = torch.tensor([3, -1, 7, 9])
    crit = ErniePretrainingCriterion(with_nsp_loss=True)
    mlm, nsp = crit(scores, rel, labels, torch.tensor([0, 1]))
    keep = labels != -1
    ref = torch.nn.functional.cross_entropy(scores[keep], labels[keep])
    assert torch.allclose(mlm, ref, atol=1e-5) and nsp > 0
    loss, _, _ = model(ids, labels=torch.full((2, 8), -100).index_fill_(1, torch.tensor([2]), 5),
                       next_sentence_label=torch.tensor([0, 1]))
    loss.backward()
    assert model.ernie.embeddings.word_embeddings.weight.grad is not None
    mlm_model = ErnieForMaskedLM(_tiny())
    assert mlm_model(ids).shape == (2, 8, 96)
    mc = ErnieForMultipleChoice(_tiny(), num_choices=3)
    logits = mc(torch.randint(1, 96, (2, 3, 8)))
    assert logits.shape == (2, 3)


def test_mlm_mask_statistics():
    g = torch.Generator().manual_seed(0)
    toks = torch.randint(1, 1000, (64, 512), generator=g)
    inp, lab = mlm_mask(toks, 1000, 999, 0.15, special_ids=(0,), generator=g)
    sel = lab >= 0
    frac = sel.float().mean().item()
    assert 0.14 < frac < 0.16
    assert torch.equal(lab[sel], toks[sel])
    masked = (inp[sel] == 999).float().mean().item()
    assert 0.77 < masked < 0.83
    assert torch.equal(inp[~sel], toks[~sel])


def test_ernie_pretrain_end_to_end(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import train as train_tool
    cfgp = os.path.join(ROOT, "fleetx_amd/configs/nlp/ernie/pretrain_ernie_base_synthetic_dp8.yaml")
    ov = ["Global.device=cpu", "Global.local_batch_size=4", "Global.micro_batch_size=4",
          "Engine.max_steps=3", "Engine.logging_freq=1", "Model.vocab_size=128",
          "Model.hidden_size=32", "Model.num_hidden_layers=2", "Model.num_attention_heads=2",
          "Model.intermediate_size=64", "Data.Train.dataset.max_seq_len=32",
          "Data.Train.dataset.vocab_size=128", "Data.Train.loader.num_workers=0",
          "Engine.save_load.output_dir=%s" % tmp_path]
    eng = train_tool.main(["-c", cfgp] + sum([["-o", o] for o in ov], []))
    assert eng is not None


def _pair_corpus(tmp_path):
    """Sentence-split corpus through the offline preprocessor (GPT BPE ids)."""
    import json
    from tests.test_generation import _tiny_bpe
    from fleetx_amd.data.data_tools.gpt import preprocess_data as P
    rs = __import__("random").Random(0)
    words = ["hello", "world", "there", "one", "two", "three", "ab", "cd"]
    lines = []
    for d in range(30):
        sents = [" ".join(rs.choice(words) for _ in range(rs.randint(2, 6))) + "."
                 for _ in range(rs.randint(2, 5))]
        lines.append(json.dumps({"text": " ".join(sents)}))
    (tmp_path / "c.jsonl").write_text("\n".join(lines) + "\n")
    tok = _tiny_bpe(tmp_path / "tok")
    prefix = str(tmp_path / "data" / "corpus")
    P.main(["--model_name", str(tok), "--tokenizer_name", "GPTTokenizer", "--input_path",
            str(tmp_path / "c.jsonl"), "--output_prefix", prefix, "--split_sentences"])
    return tmp_path / "data"


def test_ernie_sentence_pair_dataset(tmp_path):
    from fleetx_amd.data.dataset import ErnieDataset
    data = _pair_corpus(tmp_path)
    ds = ErnieDataset(str(data), [1, 0, 0], 48, 200, "Train", seed=7, cls_id=509, sep_id=510,
                      pad_id=0)
    assert len(ds) > 0
    nsp = []
    for i in range(len(ds)):
        toks, types, label, n = ds[i]
        n = int(n)
        assert toks[0] == 509 and toks[n - 1] == 510 and (toks[:n] == 510).sum() == 2
        assert (toks[n:] == 0).all() and n <= 48
        sep = int(np.nonzero(toks[:n] == 510)[0][0])
        assert (types[:sep + 1] == 0).all() and (types[sep + 1:n] == 1).all()
        nsp.append(int(label))
    assert 0.2 < np.mean(nsp) < 0.8
    a, b = ds[3], ErnieDataset(str(data), [1, 0, 0], 48, 200, "Train", seed=7, cls_id=509,
                                   sep_id=510, pad_id=0)[3]
    assert all(np.array_equal(x, y) for x, y in zip(a, b))  # deterministic per index


def test_ernie_pretrain_with_nsp(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import train as train_tool
    data = _pair_corpus(tmp_path)
    cfgp = os.path.join(ROOT, "fleetx_amd/configs/nlp/ernie/pretrain_ernie_base_synthetic_dp8.yaml")
    ov = ["Global.device=cpu", "Global.local_batch_size=4", "Global.micro_batch_size=4",
          "Engine.max_steps=3", "Engine.logging_freq=1", "Model.vocab_size=512",
          "Model.hidden_size=32", "Model.num_hidden_layers=2", "Model.num_attention_heads=2",
          "Model.intermediate_size=64", "Data.Train.dataset.name=ErnieDataset",
          "Data.Train.dataset.cls_id=509", "Data.Train.dataset.sep_id=510",
          "Data.Train.dataset.input_dir=%s" % data, "Data.Train.dataset.split=[1,0,0]",
          "Data.Train.dataset.max_seq_len=32", "Data.Train.loader.num_workers=0",
          "Data.Eval=None", "Engine.save_load.output_dir=%s" % tmp_path]
    eng = train_tool.main(["-c", cfgp] + sum([["-o", o] for o in ov], []))
    assert eng._module.pair_data and eng._module.criterion.with_nsp_loss
