"""Config system: _base_ inheritance, -o overrides, derived values
(reference ``ppfleetx/utils/config.py:30-117,163-310``)."""
import os

import pytest

from fleetx_amd.utils import config as C

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt")


def test_base_inheritance_and_derived():
    cfg = C.get_config(os.path.join(CFG, "pretrain_gpt_345M_single_card.yaml"), nranks=1)
    assert cfg.Model.hidden_size == 1024 and cfg.Model.num_layers == 24
    assert cfg.Optimizer.name == "FusedAdamW"          # from base
    assert cfg.Global.global_batch_size == 8
    assert cfg.Engine.accumulate_steps == 1
    assert cfg.Engine.test_iters == 100
    assert cfg.Distributed.dp_degree == 1


def test_override_types_and_new_keys():
    cfg = C.get_config(os.path.join(CFG, "pretrain_gpt_345M_single_card.yaml"),
                       overrides=["Model.hidden_size=512", "Optimizer.lr.max_lr=1.0/255.0",
                                  "Data.Train.dataset.split=[1,1,1]", "Engine.new_key=True",
                                  "Global.micro_batch_size=2"], nranks=1)
    assert cfg.Model.hidden_size == 512
    assert abs(cfg.Optimizer.lr.max_lr - 1.0 / 255.0) < 1e-12
    assert cfg.Data.Train.dataset.split == [1, 1, 1]
    assert cfg.Engine.new_key is True
    assert cfg.Engine.accumulate_steps == 4


def test_dp_derived_from_world():
    cfg = C.get_config(os.path.join(CFG, "pretrain_gpt_6.7B_sharding16.yaml"), nranks=32)
    assert cfg.Distributed.dp_degree == 2
    assert cfg.Global.global_batch_size == 8 * 2 * 16


def test_mismatch_adjusts_dp():
    cfg = C.get_config(os.path.join(CFG, "pretrain_gpt_1.3B_dp8.yaml"), nranks=4)
    assert cfg.Distributed.dp_degree == 4


def test_bad_batch_raises():
    with pytest.raises(AssertionError):
        C.get_config(os.path.join(CFG, "pretrain_gpt_345M_single_card.yaml"),
                     overrides=["Global.micro_batch_size=3"], nranks=1)


def test_inherited_false(tmp_path):
    base = tmp_path / "base.yaml"
    base.write_text("A:\n  x: 1\n  y: 2\nB: 3\n")
    child = tmp_path / "child.yaml"
    child.write_text("_base_: ./base.yaml\nA:\n  _inherited_: False\n  z: 5\n")
    cfg = C.parse_config(str(child))
    assert dict(cfg.A) == {"z": 5} and cfg.B == 3


def test_literal_eval_strings(tmp_path):
    f = tmp_path / "c.yaml"
    f.write_text("A:\n  v: '[1, 2]'\n  s: hello\n")
    cfg = C.parse_config(str(f))
    assert cfg.A.v == [1, 2] and cfg.A.s == "hello"


def test_auto_config():
    p = os.path.join(CFG, "auto", "pretrain_gpt_1.3B_dp8.yaml")
    if not os.path.exists(p):
        pytest.skip("auto configs not present")
    cfg = C.get_auto_config(p, nranks=8)
    assert cfg.Distributed.dp_degree == 8
    assert "strategy" in cfg.Engine
