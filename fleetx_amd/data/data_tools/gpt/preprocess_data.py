"""Offline GPT corpus preprocessing: jsonl documents -> ``<prefix>_ids.npy`` +
``<prefix>_idx.npz``, the input format of :class:`GPTDataset`.

    python -m fleetx_amd.data.data_tools.gpt.preprocess_data \\
        --model_name ./gpt2-tokenizer --tokenizer_name GPTTokenizer \\
        --input_path corpus.jsonl --output_prefix data/corpus --append_eos --workers 40

Parity: reference ``ppfleetx/data/data_tools/gpt/preprocess_data.py`` (D12,
SURVEY §2.6): the same command line (``--model_name --tokenizer_name
--input_path --output_prefix --json_key --split_sentences --append_eos
--workers --log_interval`` and the Chinese whole-word-mask switches) and the
same output contract -- token ids as ``uint16`` when the vocabulary has fewer
than 65535 entries, else ``int32``; ``idx.npz`` with ``lens`` (int32 tokens per
sentence) and ``docs`` (int64 cumulative sentence count per document, leading
0).

Design: a worker pool tokenizes documents while the parent streams the ids to
a raw side file (the reference held the whole corpus in a ``BytesIO``, i.e.
RAM >= corpus size); the final ``.npy`` is a header plus a chunked copy of
that file.  Offline only: tokenizers load from a local directory, and without
nltk's punkt model English sentences are split by a punctuation regex.
"""
import argparse
import json
import multiprocessing
import os
import re
import sys
import time

import numpy as np

_SENT_RE = re.compile(r"(?<=[.!?。！？])\s+")
_CJK_RE = re.compile("[一-龥]")


def get_args(argv=None):
    ap = argparse.ArgumentParser(description="jsonl -> GPTDataset ids/idx files")
    ap.add_argument("--model_name", required=True,
                    help="local tokenizer directory (vocab.json+merges.txt, or vocab.txt)")
    ap.add_argument("--tokenizer_name", required=True,
                    choices=["GPTTokenizer", "GPTChineseTokenizer", "ErnieTokenizer",
                             "BertTokenizer", "ElectraTokenizer"])
    g = ap.add_argument_group("data input/output")
    g.add_argument("--input_path", required=True, help="a .jsonl file or a directory of them")
    g.add_argument("--output_prefix", required=True)
    g.add_argument("--data_format", default="JSON", choices=["JSON"])
    g.add_argument("--json_key", default="text")
    g.add_argument("--split_sentences", action="store_true")
    g = ap.add_argument_group("chinese words")
    g.add_argument("--chinese", action="store_true")
    g.add_argument("--cn_whole_word_segment", action="store_true")
    g.add_argument("--cn_seg_func", default="jieba", choices=["lac", "seg", "jieba"])
    g.add_argument("--cn_splited", action="store_true",
                   help="the corpus is already segmented into words")
    g.add_argument("--cn_split_dimer", default=" ")
    g = ap.add_argument_group("common config")
    g.add_argument("--append_eos", action="store_true")
    g.add_argument("--log_interval", type=int, default=100)
    g.add_argument("--workers", type=int, default=1)
    return ap.parse_args(argv)


class _WordPiece:
    """Adapter giving a WordPiece vocabulary the GPTTokenizer surface."""

    def __init__(self, vocab_file):
        from transformers import BertTokenizer
        self.tok = BertTokenizer(vocab_file)

    def tokenize(self, text):
        return self.tok.tokenize(text)

    def convert_tokens_to_ids(self, tokens):
        return self.tok.convert_tokens_to_ids(tokens)

    @property
    def vocab_size(self):
        return self.tok.vocab_size

    @property
    def eos_token_id(self):
        return self.tok.sep_token_id


def load_tokenizer(name, model_name):
    if name in ("GPTTokenizer", "GPTChineseTokenizer"):
        from fleetx_amd.data.tokenizers import GPTTokenizer
        return GPTTokenizer.from_pretrained(model_name)
    vocab = os.path.join(model_name, "vocab.txt") if os.path.isdir(model_name) else model_name
    if not os.path.isfile(vocab):
        raise FileNotFoundError("{} needs a local WordPiece vocab.txt (got {}); this toolkit "
                                "never downloads".format(name, model_name))
    return _WordPiece(vocab)


def whole_word_mask_tokens(tokens, words, max_word_length=4):
    """Prefix the non-initial characters of multi-character Chinese words with
    ``##`` so whole-word masking treats the word as one unit (reference
    ``get_whole_word_mask_tokens``)."""
    words = set(words)
    out, i = [], 0
    while i < len(tokens):
        if not _CJK_RE.search(tokens[i]):
            out.append(tokens[i])
            i += 1
            continue
        for n in range(min(max_word_length, len(tokens) - i), 0, -1):
            if n == 1 or "".join(tokens[i:i + n]) in words:
                out.append(tokens[i])
                out.extend("##" + t for t in tokens[i + 1:i + n])
                i += n
                break
    return out


def _english_splitter():
    try:
        import nltk
        punkt = nltk.data.load("tokenizers/punkt/english.pickle")
        return punkt.tokenize
    except Exception:  # no nltk or no punkt model offline: punctuation regex
        return lambda text: [s for s in _SENT_RE.split(text) if s]


def _segmenter(name):
    if name == "jieba":
        try:
            import jieba
        except ImportError as e:
            raise ImportError("--cn_seg_func jieba needs the jieba package (not installed); "
                              "pre-segment the corpus and pass --cn_splited") from e
        return lambda text: list(jieba.cut(text))
    try:
        from LAC import LAC
    except ImportError as e:
        raise ImportError("--cn_seg_func {} needs the LAC package (not installed); pre-segment "
                          "the corpus and pass --cn_splited".format(name)) from e
    lac = LAC(mode="lac" if name == "lac" else "seg")
    return lambda text: lac.run(text)[0] if name == "lac" else lac.run(text)


class Converter:
    """Per-worker tokenization state (created by the pool initializer)."""

    def __init__(self, args):
        self.args = args

    def initializer(self):
        a = self.args
        Converter.tokenizer = load_tokenizer(a.tokenizer_name, a.model_name)
        if a.split_sentences:
            Converter.split = (lambda t: t.split("\n")) if a.chinese else _english_splitter()
        else:
            Converter.split = lambda t: [t]
        if a.cn_whole_word_segment:
            Converter.segment = (lambda t: t.split(a.cn_split_dimer)) if a.cn_splited \
                else _segmenter(a.cn_seg_func)
            Converter.wwm = staticmethod(whole_word_mask_tokens)
        else:
            Converter.segment = lambda t: t
            Converter.wwm = staticmethod(lambda toks, words: toks)

    @staticmethod
    def process(text):
        words = Converter.segment(text)
        tokens = Converter.tokenizer.tokenize("".join(words))
        tokens = Converter.wwm(tokens, words)
        return Converter.tokenizer.convert_tokens_to_ids(tokens)

    def encode(self, json_line):
        text = json.loads(json_line)[self.args.json_key]
        doc = []
        for sentence in Converter.split(text):
            ids = Converter.process(sentence.strip())
            if ids:
                doc.append(ids)
        if doc and self.args.append_eos:
            doc[-1].append(Converter.tokenizer.eos_token_id)
        return doc, len(text.encode("utf-8"))


def _input_files(path):
    if os.path.isfile(path):
        return [path]
    return sorted(os.path.join(r, f) for r, _, fs in os.walk(path) for f in fs)


def main(argv=None):
    args = get_args(argv)
    files = _input_files(args.input_path)
    if not files:
        raise SystemExit("No input file found!")
    tok = load_tokenizer(args.tokenizer_name, args.model_name)
    dtype = np.uint16 if tok.vocab_size < 65535 else np.int32
    conv = Converter(args)
    pool = None
    if args.workers > 1:
        pool = multiprocessing.Pool(args.workers, initializer=conv.initializer)
    else:
        conv.initializer()
    raw_path = args.output_prefix + "_ids.raw.tmp"
    os.makedirs(os.path.dirname(os.path.abspath(raw_path)), exist_ok=True)
    lens, docs = [], [0]
    n_tokens, step, nbytes, t0 = 0, 0, 0, time.time()
    try:
        with open(raw_path, "wb") as raw:
            for path in files:
                if not path.endswith((".jsonl", ".json")):
                    print("Unexpected data format, skipped %s" % path, file=sys.stderr)
                    continue
                with open(path, "r", encoding="utf-8") as fin:
                    lines = (l for l in fin if l.strip())
                    it = pool.imap(conv.encode, lines, 256) if pool else map(conv.encode, lines)
                    for doc, nb in it:
                        step += 1
                        nbytes += nb
                        if not doc:
                            continue
                        for sent in doc:
                            raw.write(np.asarray(sent, dtype=dtype).tobytes())
                            lens.append(len(sent))
                            n_tokens += len(sent)
                        docs.append(len(lens))
                        if step % args.log_interval == 0:
                            el = time.time() - t0
                            print("Processed %d documents (%.2f docs/s, %.4f MB/s)."
                                  % (step, step / el, nbytes / el / 2 ** 20), file=sys.stderr)
    finally:
        if pool is not None:
            pool.close()
            pool.join()
    out = np.lib.format.open_memmap(args.output_prefix + "_ids.npy", mode="w+", dtype=dtype,
                                    shape=(n_tokens,))
    if n_tokens:
        src = np.memmap(raw_path, dtype=dtype, mode="r", shape=(n_tokens,))
        for i in range(0, n_tokens, 1 << 26):
            out[i:i + (1 << 26)] = src[i:i + (1 << 26)]
        del src
    out.flush()
    del out
    os.remove(raw_path)
    np.savez(args.output_prefix + "_idx.npz", lens=np.asarray(lens, dtype=np.int32),
             docs=np.asarray(docs, dtype=np.int64))
    nsent, ndoc = len(lens), len(docs) - 1
    print("Total sentences num: %d" % nsent)
    print("Total documents num: %d" % ndoc)
    print("Total tokens num: %d" % n_tokens)
    if nsent and ndoc:
        print("Average tokens per sentence: %.2f" % (n_tokens / nsent))
        print("Average tokens per document: %.2f" % (n_tokens / ndoc))
    return n_tokens


if __name__ == "__main__":
    main()
