"""Generation (KV-cache decode vs full recompute), logits processors,
sampling filters, and the offline BPE tokenizer (reference C20/C27, D08)."""
import json

import pytest
import torch

from fleetx_amd.models.language_model.gpt.model import GPTConfig, GPTForPretraining
from fleetx_amd.models.language_model.gpt import generation as G


def _model(seed=0):
    torch.manual_seed(seed)
    cfg = GPTConfig(vocab_size=97, hidden_size=64, num_layers=2, num_attention_heads=4,
                    max_position_embeddings=64, hidden_dropout_prob=0.0,
                    attention_probs_dropout_prob=0.0)
    m = GPTForPretraining(cfg)
    with torch.no_grad():  # non-trivial LN/bias so the check is meaningful
        for n, p in m.named_parameters():
            if p.ndim == 1:
                p.add_(0.05 * torch.randn_like(p))
    return m.eval()


def _naive_greedy(model, ids, n):
    out = []
    cur = ids
    for _ in range(n):
        with torch.no_grad():
            logits = model(cur)
        nxt = logits[:, -1].argmax(-1)
        out.append(nxt)
        cur = torch.cat([cur, nxt[:, None]], 1)
    return torch.stack(out, 1)


def test_greedy_cached_matches_recompute():
    m = _model()
    gen = G.GPTForGeneration(m, {"decode_strategy": "greedy_search", "max_dec_len": 8,
                                 "eos_token_id": None})
    ids = torch.randint(0, 97, (2, 5))
    out, scores = gen.generate(ids)
    ref = _naive_greedy(m, ids, 8)
    assert torch.equal(out, ref)
    assert scores.shape == (2,)


def test_ragged_prompts_use_lengths():
    m = _model(1)
    gen = G.GPTForGeneration(m, {"decode_strategy": "greedy_search", "max_dec_len": 4,
                                 "eos_token_id": None})
    a = torch.randint(0, 97, (1, 7))
    b = torch.randint(0, 97, (1, 4))
    batch = torch.cat([a, torch.cat([b, torch.zeros(1, 3, dtype=torch.long)], 1)])
    out, _ = gen.generate(batch, torch.tensor([7, 4]))
    assert torch.equal(out[0], _naive_greedy(m, a, 4)[0])
    assert torch.equal(out[1], _naive_greedy(m, b, 4)[0])


def test_sampling_eos_stops_and_pads():
    m = _model(2)
    gen = G.GPTForGeneration(m, {"decode_strategy": "sampling", "top_k": 5, "top_p": 0.9,
                                 "temperature": 0.7, "max_dec_len": 10, "eos_token_id": 3,
                                 "pad_token_id": 0, "min_dec_len": 2})
    out, _ = gen.generate(torch.randint(4, 97, (3, 6)), seed=5)
    assert out.shape[0] == 3 and out.shape[1] <= 10
    assert not (out[:, :2] == 3).any()  # min length respected
    for row in out.tolist():
        if 3 in row:
            assert all(t == 0 for t in row[row.index(3) + 1:])


def test_filters_and_processors():
    probs = torch.tensor([[0.5, 0.3, 0.15, 0.05]])
    assert torch.equal(G.top_k_filter(probs, 2) > 0, torch.tensor([[True, True, False, False]]))
    kept = G.top_p_filter(probs, 0.7) > 0
    assert kept.tolist() == [[True, True, False, False]]
    lg = torch.tensor([[2.0, -2.0, 1.0]])
    out = G.RepetitionPenaltyLogitsProcessor(2.0)(torch.tensor([[0, 1]]), lg.clone())
    assert out.tolist() == [[1.0, -4.0, 1.0]]
    f = G.ForcedBOSTokenLogitsProcessor(2)
    o = f(None, torch.zeros(1, 3))
    assert o.argmax().item() == 2


def _tiny_bpe(tmp_path):
    from fleetx_amd.data.tokenizers import bytes_to_unicode
    tmp_path.mkdir(parents=True, exist_ok=True)
    base = list(bytes_to_unicode().values())
    vocab = {c: i for i, c in enumerate(base)}
    merges = [("h", "e"), ("l", "l"), ("he", "ll"), ("Ġ", "w")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    vocab["<|endoftext|>"] = len(vocab)
    (tmp_path / "vocab.json").write_text(json.dumps(vocab))
    (tmp_path / "merges.txt").write_text("#version: 0.2\n" + "\n".join("%s %s" % m for m in merges))
    return tmp_path


def test_tokenizer_roundtrip(tmp_path):
    from fleetx_amd.data.tokenizers import GPTTokenizer
    tok = GPTTokenizer.from_pretrained(str(_tiny_bpe(tmp_path)))
    text = "hello world! ünïcödé 123"
    ids = tok.encode(text)
    assert tok.decode(ids) == text
    assert tok.tokenize("hello")[0] == "hell"
    assert tok.eos_token_id == len(tok.encoder) - 1


def test_tokenizer_missing_files_is_clear(tmp_path, monkeypatch):
    from fleetx_amd.data.tokenizers import GPTTokenizer
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.delenv("FLEETX_TOKENIZER_DIR", raising=False)
    with pytest.raises(FileNotFoundError):
        GPTTokenizer.from_pretrained("gpt2")
