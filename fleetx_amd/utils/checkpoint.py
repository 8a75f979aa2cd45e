"""Checkpoint layout and atomic IO.

Layout parity with reference ``eager_engine.py:581-660`` (§5.4):

    <output_dir>/epoch_{E}_step_{S}/[mp_{MP:02d}_sharding_{SH:02d}_pp_{PP:02d}/]
        model.pdparams      model state dict (model dtype)
        model_state.pdopt   optimizer state (fp32 master, moments, LR state)
        meta_state.pdopt    {epoch, step, consumed_samples, rng tracker, scaler}

Payloads are plain tensor dicts written with ``torch.save`` and read with
``torch.load(weights_only=True)``.  Writes go to a temp directory that is
renamed into place, so a crash never leaves a half-written checkpoint.
"""
import os
import shutil

import torch


def shard_dirname(mp_rank, sharding_rank, pp_rank):
    return "mp_{:0>2d}_sharding_{:0>2d}_pp_{:0>2d}".format(mp_rank, sharding_rank, pp_rank)


def step_dir(output_dir, epoch, step):
    return os.path.join(output_dir, "epoch_{}_step_{}".format(epoch, step))


def save_payloads(target_dir, payloads):
    """payloads: {filename: object}; atomic directory publish."""
    parent = os.path.dirname(target_dir.rstrip("/")) or "."
    os.makedirs(parent, exist_ok=True)
    tmp = target_dir.rstrip("/") + ".tmp.%d" % os.getpid()
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    os.makedirs(tmp)
    for name, obj in payloads.items():
        torch.save(obj, os.path.join(tmp, name))
    if os.path.exists(target_dir):
        shutil.rmtree(target_dir)
    os.replace(tmp, target_dir)


def load_payload(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def _complete(step_path, shards):
    """Every expected shard directory has its meta file (written last)."""
    if not shards:
        return os.path.isfile(os.path.join(step_path, "meta_state.pdopt")) or any(
            os.path.isfile(os.path.join(step_path, d, "meta_state.pdopt"))
            for d in os.listdir(step_path) if d.startswith("mp_"))
    return all(os.path.isfile(os.path.join(step_path, d, "meta_state.pdopt")) for d in shards)


def latest_checkpoint(output_dir, shards=None):
    """Most recent COMPLETE ``epoch_E_step_S`` directory (automatic resume).

    ``shards``: the shard directory names every (mp, sharding, pp) rank
    writes; a step directory missing any of them (a crash mid-save) is
    skipped in favour of the previous one."""
    if not os.path.isdir(output_dir):
        return None
    cands = []
    for d in os.listdir(output_dir):
        if d.startswith("epoch_") and "_step_" in d and ".tmp" not in d:
            try:
                e, s = d[len("epoch_"):].split("_step_")
                cands.append(((int(e), int(s)), os.path.join(output_dir, d)))
            except ValueError:
                continue
    for _, path in sorted(cands, reverse=True):
        if _complete(path, shards):
            return path
    return None
