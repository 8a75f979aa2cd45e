"""Config-driven preprocessing pipelines (reference ``data/transforms/utils.py:18-43``)."""
from . import preprocess


def transform(data, ops=()):
    for op in ops:
        data = op(data)
    return data


def create_preprocess_operators(params):
    """``[{OpName: {kwargs}}, ...]`` -> list of operator instances."""
    assert isinstance(params, (list, tuple)), "operator config should be a list"
    ops = []
    for item in params:
        assert isinstance(item, dict) and len(item) == 1, "yaml format error"
        name = list(item)[0]
        kwargs = item[name] or {}
        if not hasattr(preprocess, name) or name.startswith("_"):
            raise ValueError("unknown preprocess operator {}".format(name))
        ops.append(getattr(preprocess, name)(**dict(kwargs)))
    return ops
