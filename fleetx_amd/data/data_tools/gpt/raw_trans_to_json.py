"""Raw text corpus -> jsonl (one ``{json_key: document}`` object per line),
the input of :mod:`preprocess_data`.

    python -m fleetx_amd.data.data_tools.gpt.raw_trans_to_json \\
        --input_path raw_dir --output_path corpus --workers 8

Parity: reference ``ppfleetx/data/data_tools/gpt/raw_trans_to_json.py`` (D12):
documents are separated by lines equal to ``--doc_spliter`` (blank by
default), documents of at most ``--min_doc_length`` characters are dropped,
files convert in a process pool, then are merged into ``<output_path>.jsonl``
and shuffled.  The shuffle is an in-process seeded permutation (reproducible;
the reference shelled out to ``shuf``).
"""
import argparse
import json
import multiprocessing
import os
import random
import shutil
import sys
import time
from functools import partial


def get_args(argv=None):
    ap = argparse.ArgumentParser(description="raw text -> jsonl documents")
    ap.add_argument("--input_path", required=True, help="raw file or folder")
    ap.add_argument("--output_path", required=True)
    ap.add_argument("--json_key", default="text")
    ap.add_argument("--doc_spliter", default="",
                    help="separator line between documents (lines are stripped first)")
    ap.add_argument("--min_doc_length", type=int, default=10)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--log_interval", type=int, default=1)
    ap.add_argument("--no-merge", dest="no_merge", action="store_true")
    ap.add_argument("--no-shuffle", dest="no_shuffle", action="store_true")
    ap.add_argument("--seed", type=int, default=1234)
    return ap.parse_args(argv)


def raw_text_to_json(path, doc_spliter="", json_key="text", min_doc_length=10):
    """Convert one raw file to ``<path>.jsonl``; returns (bytes read, out path)."""
    path = os.path.abspath(path)
    if not os.path.exists(path):
        return 0, None
    out_path = path + ".jsonl"
    nread = 0
    with open(path, "r", encoding="utf-8") as fin, open(out_path, "w", encoding="utf-8") as fout:
        doc = []
        for line in fin:
            nread += len(line)
            if line.strip() == doc_spliter:
                text = "".join(doc)
                if len(text) > min_doc_length:
                    fout.write(json.dumps({json_key: text}, ensure_ascii=False) + "\n")
                doc = []
            else:
                doc.append(line)
        text = "".join(doc)
        if len(text) > min_doc_length:
            fout.write(json.dumps({json_key: text}, ensure_ascii=False) + "\n")
    return nread, out_path


def merge_file(paths, output_path):
    if not output_path.endswith(".jsonl"):
        output_path += ".jsonl"
    with open(output_path, "wb") as out:
        for p in paths:
            if p is not None and os.path.exists(p):
                with open(p, "rb") as f:
                    shutil.copyfileobj(f, out)
                os.remove(p)
    return output_path


def shuffle_file(path, seed=1234):
    with open(path, "r", encoding="utf-8") as f:
        lines = f.readlines()
    random.Random(seed).shuffle(lines)
    with open(path, "w", encoding="utf-8") as f:
        f.writelines(lines)


def main(argv=None):
    args = get_args(argv)
    if os.path.isfile(args.input_path):
        files = [args.input_path]
    else:
        files = sorted(os.path.join(r, f) for r, _, fs in os.walk(args.input_path) for f in fs
                       if not f.endswith(".jsonl"))
    conv = partial(raw_text_to_json, doc_spliter=args.doc_spliter, json_key=args.json_key,
                   min_doc_length=args.min_doc_length)
    t0, total, outs = time.time(), 0, []
    with multiprocessing.Pool(max(1, args.workers)) as pool:
        for i, (nb, out) in enumerate(pool.imap(conv, files, 1), start=1):
            total += nb
            outs.append(out)
            if i % args.log_interval == 0:
                el = time.time() - t0
                print("Processed %d files (%.2f files/s, %.2f MB/s)."
                      % (i, i / el, total / el / 2 ** 20), file=sys.stderr)
    if args.no_merge:
        return outs
    merged = merge_file(outs, args.output_path)
    if not args.no_shuffle:
        shuffle_file(merged, args.seed)
    print("File saved in %s" % merged)
    return merged


if __name__ == "__main__":
    main()
