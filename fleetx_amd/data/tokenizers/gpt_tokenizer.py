"""GPT-2 byte-level BPE tokenizer (offline).

Parity: reference ``ppfleetx/data/tokenizers/gpt_tokenizer.py:30-392`` (D08):
byte->unicode table, BPE merge loop with a cache, ``encode / decode /
convert_ids_to_string / tokenize / convert_tokens_to_ids``, ``eos_token_id``
(``<|endoftext|>``, 50256 for GPT-2).

Difference: no download.  ``from_pretrained(name_or_dir)``
resolves ``vocab.json`` + ``merges.txt`` from the given directory,
``$FLEETX_TOKENIZER_DIR``, ``~/.cache/fleetx_amd/<name>`` or the reference's
cache ``~/.cache/ppfleetx``; a clear error explains where to put the files.
"""
import json
import os
from functools import lru_cache

import regex as re


@lru_cache()
def bytes_to_unicode():
    """Map every byte to a printable unicode char (reversible)."""
    printable = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    table = {b: chr(b) for b in printable}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def _pairs(word):
    return {(a, b) for a, b in zip(word[:-1], word[1:])}


PAT = re.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")



# reference gpt_tokenizer.py pretrained resource URLs (vocab, merges)
PRETRAINED_URLS = {
    "gpt2": ("http://fleet.bj.bcebos.com/datasets/gpt/gpt2-vocab.json",
             "http://fleet.bj.bcebos.com/datasets/gpt/gpt2-merges.txt"),
}

class GPTTokenizer:
    eos_token = "<|endoftext|>"

    def __init__(self, vocab_file, merges_file, errors="replace", max_len=None, special_tokens=None):
        with open(vocab_file, "r", encoding="utf-8") as f:
            self.encoder = json.load(f)
        self.decoder = {v: k for k, v in self.encoder.items()}
        with open(merges_file, "r", encoding="utf-8") as f:
            lines = f.read().split("\n")
        merges = [tuple(l.split()) for l in lines if l and not l.startswith("#version")]
        merges = [m for m in merges if len(m) == 2]
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        self.errors = errors
        self.max_len = max_len or int(1e12)
        self.cache = {}
        self.special_tokens = {}
        self.special_tokens_decoder = {}
        self.set_special_tokens(special_tokens or [])

    # --------------------------------------------------------------- loading
    @classmethod
    def from_pretrained(cls, name_or_dir="gpt2", cache_dir=None, **kwargs):
        cands = []
        if os.path.isdir(str(name_or_dir)):
            cands.append(str(name_or_dir))
        if os.environ.get("FLEETX_TOKENIZER_DIR"):
            cands.append(os.environ["FLEETX_TOKENIZER_DIR"])
        if cache_dir:
            cands.append(cache_dir)
        home = os.path.expanduser("~")
        cands += [os.path.join(home, ".cache", "fleetx_amd", str(name_or_dir)),
                  os.path.join(home, ".cache", "ppfleetx")]
        for d in cands:
            v, m = os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt")
            if not os.path.exists(v):
                v = os.path.join(d, "gpt2-vocab.json")
                m = os.path.join(d, "gpt2-merges.txt")
            if os.path.exists(v) and os.path.exists(m):
                return cls(v, m, **kwargs)
        # the reference's hosted vocab (gpt_tokenizer.py:126-128) through the
        # offline cache: found if a previous run / the user put it there
        urls = PRETRAINED_URLS.get(str(name_or_dir))
        if urls is not None:
            from ...utils.download import cached_path
            try:
                return cls(cached_path(urls[0], cache_dir), cached_path(urls[1], cache_dir),
                           **kwargs)
            except (FileNotFoundError, TimeoutError):
                pass
        raise FileNotFoundError(
            "GPT-2 tokenizer files not found (looked in {}). Place vocab.json and merges.txt in "
            "one of these directories or set FLEETX_TOKENIZER_DIR; FleetX-AMD never downloads."
            .format(cands))

    # --------------------------------------------------------------- specials
    def set_special_tokens(self, special_tokens):
        if not special_tokens:
            return
        self.special_tokens = {t: len(self.encoder) + i for i, t in enumerate(special_tokens)}
        self.special_tokens_decoder = {v: k for k, v in self.special_tokens.items()}

    def __len__(self):
        return len(self.encoder) + len(self.special_tokens)

    @property
    def vocab_size(self):
        return len(self.encoder)

    @property
    def eos_token_id(self):
        return self.encoder[self.eos_token]

    @property
    def eod(self):
        return self.eos_token_id

    # --------------------------------------------------------------- BPE
    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token)
        pairs = _pairs(word)
        if not pairs:
            return token
        while True:
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            first, second = best
            out, i = [], 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    out.extend(word[i:])
                    break
                out.extend(word[i:j])
                i = j
                if word[i] == first and i < len(word) - 1 and word[i + 1] == second:
                    out.append(first + second)
                    i += 2
                else:
                    out.append(word[i])
                    i += 1
            word = tuple(out)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        res = " ".join(word)
        self.cache[token] = res
        return res

    def tokenize(self, text):
        toks = []
        for t in PAT.findall(text):
            t = "".join(self.byte_encoder[b] for b in t.encode("utf-8"))
            toks.extend(self.bpe(t).split(" "))
        return toks

    def convert_tokens_to_ids(self, tokens):
        if isinstance(tokens, str):
            return self.special_tokens.get(tokens, self.encoder.get(tokens, 0))
        return [self.special_tokens.get(t, self.encoder.get(t, 0)) for t in tokens]

    def convert_ids_to_tokens(self, ids, skip_special_tokens=False):
        out = []
        for i in ids:
            if i in self.special_tokens_decoder:
                if not skip_special_tokens:
                    out.append(self.special_tokens_decoder[i])
            else:
                out.append(self.decoder[i])
        return out

    def encode(self, text):
        return self.convert_tokens_to_ids(self.tokenize(text))

    def decode(self, ids):
        text = "".join(self.decoder[int(i)] for i in ids)
        return bytearray([self.byte_decoder[c] for c in text]).decode("utf-8", errors=self.errors)

    def convert_ids_to_string(self, ids):
        return self.decode(ids)

    def __call__(self, text):
        return {"input_ids": self.encode(text)}
