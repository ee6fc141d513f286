"""Drop-in import name of the reference package.

``import news_rec_utils.data_model_helper`` (and every other submodule the
reference scripts import) resolves to the MI355X implementation in
``news_recommendation_project_v2_amd``: each submodule is aliased in
``sys.modules`` so module identity (and isinstance checks) is preserved.
"""
import importlib
import sys

_PKG = "news_recommendation_project_v2_amd"
_SUBMODULES = ("config", "attention", "data_utils", "modeling_utils", "latent_attention", "data_model_helper", "evaluation",
               "pipeline", "components", "trainer", "engine", "ops", "synthetic", "weights")

for _name in _SUBMODULES:
    _mod = importlib.import_module(f"{_PKG}.{_name}")
    sys.modules[f"{__name__}.{_name}"] = _mod
    globals()[_name] = _mod
