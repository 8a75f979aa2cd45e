"""Offline data pipeline (reference D12/D13): raw text -> jsonl -> ids/idx
files that GPTDataset reads, Chinese whole-word-mask marking, and the
multi-process shell-command tool."""
import json
import os
import sys

import numpy as np

from tests.test_generation import _tiny_bpe


def test_raw_to_json_to_ids_roundtrip(tmp_path):
    from fleetx_amd.data.data_tools.gpt import raw_trans_to_json as R
    from fleetx_amd.data.data_tools.gpt import preprocess_data as P
    from fleetx_amd.data.tokenizers import GPTTokenizer
    raw = tmp_path / "raw"
    raw.mkdir()
    (raw / "a.txt").write_text("hello world. hello there!\n\nshort\n\nworld hello world\n")
    (raw / "b.txt").write_text("the second file has one longer document\n")
    merged = R.main(["--input_path", str(raw), "--output_path", str(tmp_path / "corpus"),
                     "--workers", "2", "--min_doc_length", "6"])
    docs = [json.loads(l)["text"] for l in open(merged)]
    assert sorted(docs) == sorted(["hello world. hello there!\n", "world hello world\n",
                                   "the second file has one longer document\n"])
    tokdir = _tiny_bpe(tmp_path / "tok")
    prefix = str(tmp_path / "out" / "corpus")
    n = P.main(["--model_name", str(tokdir), "--tokenizer_name", "GPTTokenizer",
                "--input_path", merged, "--output_prefix", prefix, "--split_sentences",
                "--append_eos", "--workers", "2", "--log_interval", "1"])
    ids = np.load(prefix + "_ids.npy")
    idx = np.load(prefix + "_idx.npz")
    tok = GPTTokenizer.from_pretrained(str(tokdir))
    assert ids.dtype == np.uint16 and len(ids) == n == idx["lens"].sum()
    assert idx["docs"].dtype == np.int64 and idx["lens"].dtype == np.int32
    assert idx["docs"][0] == 0 and len(idx["docs"]) == 4
    # every document ends with EOS; sentences decode back to the text
    ends = np.cumsum(idx["lens"])[idx["docs"][1:] - 1]
    assert all(ids[e - 1] == tok.eos_token_id for e in ends)
    by_doc = []
    for d in range(3):
        s0 = int(np.sum(idx["lens"][:idx["docs"][d]]))
        s1 = int(np.sum(idx["lens"][:idx["docs"][d + 1]]))
        by_doc.append(tok.decode([int(t) for t in ids[s0:s1 - 1]]))
    assert any(t.startswith("hello world.") and "hello there!" in t for t in by_doc)


def test_whole_word_mask_marks_inner_characters():
    from fleetx_amd.data.data_tools.gpt.preprocess_data import whole_word_mask_tokens
    toks = ["通", "过", "利", "用", "me", "##rc", "核", "，"]
    out = whole_word_mask_tokens(toks, ["通过", "利用", "mercer", "核", "，"])
    assert out == ["通", "##过", "利", "##用", "me", "##rc", "核", "，"]


def test_multiprocess_tool(tmp_path):
    from fleetx_amd.tools import multiprocess_tool as M
    lst = tmp_path / "cmds.txt"
    cmds = ["echo %d > %s" % (i, tmp_path / ("o%d" % i)) for i in range(6)]
    lst.write_text("# comment\n" + "\n".join(cmds) + "\n\nexit 3\n")
    rc = M.main(["--num_proc", "3", "--shell_cmd_list_filename", str(lst)])
    assert rc == 1  # the `exit 3` line failed and is reported
    assert all((tmp_path / ("o%d" % i)).read_text().strip() == str(i) for i in range(6))
