"""Module registry (reference ``ppfleetx/models/__init__.py:28-32``: ``eval(Model.module)``).

Modules register by name; ``build_module`` looks the name up instead of
evaluating it.
"""
from ..core.module.basic_module import BasicModule

_MODULES = {}


def register_module(name):
    def deco(cls):
        _MODULES[name] = cls
        return cls
    return deco


def _lazy_defaults():
    if _MODULES:
        return
    from .language_model.language_module import GPTModule
    _MODULES["GPTModule"] = GPTModule
    _MODULES["BasicModule"] = BasicModule
    try:
        from .language_model.language_module import GPTGenerationModule, GPTEvalModule
        _MODULES["GPTGenerationModule"] = GPTGenerationModule
        _MODULES["GPTEvalModule"] = GPTEvalModule
    except ImportError:
        pass
    for modname, names in (("language_model.gpt.auto.auto_module", ["GPTModuleAuto"]),
                           ("language_model.ernie.ernie_module", ["ErnieModule"]),
                           ("vision_model.general_classification_module", ["GeneralClsModule"]),
                           ("multimodal_model.multimodal_module", ["ImagenModule"])):
        try:
            mod = __import__("fleetx_amd.models." + modname, fromlist=names)
        except ImportError:
            continue
        for n in names:
            if hasattr(mod, n):
                _MODULES[n] = getattr(mod, n)


def build_module(config):
    _lazy_defaults()
    name = config.Model.get("module", "BasicModule")
    if name not in _MODULES:
        raise ValueError("unknown module {} (known: {})".format(name, sorted(_MODULES)))
    return _MODULES[name](config)
