"""Named-step pipeline over train/val context dicts (reference pipeline.py:1-90).

Same API (``Pipeline(name, steps).transform(ctx, val_ctx)``,
``PipelineComponent.transform/train``, ``check_req_keys``).  One deliberate
difference: the reference caches each step's output under
``cache/{name}_{step}.pkl.gz`` keyed by name only (pipeline.py:55-74), so a
stale cache from another run is silently reused.  Here caching is
off by default and, when on, the cache key includes a digest of the input
context so a different input never hits an old entry.
"""
from __future__ import annotations

import hashlib
from abc import ABC, abstractmethod
from pathlib import Path
from typing import Any, Iterable, Optional


def check_req_keys(required_keys: set[str], context_dict: dict[str, Any]) -> None:
    for key in required_keys:
        assert key in context_dict, f"Required Key {key} is not present in context_dict"


class PipelineComponent(ABC):
    required_keys: set = set()
    train_required_keys: set = set()

    @abstractmethod
    def transform(self, context_dict: dict[str, Any]) -> dict[str, Any]:
        ...

    def train(self, context_dict: dict[str, Any], val_context_dict: Optional[dict[str, Any]] = None) -> None:
        pass


def _digest(ctx: Optional[dict]) -> str:
    if not ctx:
        return "none"
    h = hashlib.sha1()
    for k in sorted(ctx):
        h.update(k.encode())
        v = ctx[k]
        try:
            import numpy as np
            import torch
            if isinstance(v, torch.Tensor):
                h.update(str(tuple(v.shape)).encode())
                h.update(v.detach().flatten()[:4096].cpu().numpy().tobytes())
            elif isinstance(v, np.ndarray) and v.dtype != object:
                h.update(str(v.shape).encode())
                h.update(v.ravel()[:65536].tobytes())
            else:
                h.update(repr(type(v)).encode())
                h.update(repr(v)[:65536].encode())
        except Exception:  # unhashable exotic value: key by type only
            h.update(repr(type(v)).encode())
    return h.hexdigest()[:16]


class Pipeline:
    def __init__(self, name: str, steps: Iterable[tuple[str, PipelineComponent]], use_cache: bool = False,
                 cache_dir: Path = Path("cache")):
        self.name = name
        self._steps = list(steps)
        self.use_cache = use_cache
        self.cache_dir = Path(cache_dir)
        if use_cache:
            self.cache_dir.mkdir(parents=True, exist_ok=True)

    def _iterate_over_steps(self, context_dict, val_context_dict=None, training: bool = False):
        for step_name, component in self._steps:
            print(f"Starting step {step_name}")
            cache_file = None
            if self.use_cache:
                import joblib
                key = _digest(context_dict) + _digest(val_context_dict)
                cache_file = self.cache_dir / f"{self.name}_{step_name}_{key}.pkl.gz"
                if cache_file.is_file():
                    loaded = joblib.load(cache_file)
                    context_dict, val_context_dict = loaded["context_dict"], loaded["val_context_dict"]
                    print(f"Completed step {step_name} (cached)")
                    continue
            if training:
                component.train(context_dict, val_context_dict)
            context_dict = component.transform(context_dict)
            if val_context_dict:
                val_context_dict = component.transform(val_context_dict)
            if cache_file is not None:
                import joblib
                joblib.dump({"context_dict": context_dict, "val_context_dict": val_context_dict}, cache_file,
                            compress=True)
            print(f"Completed step {step_name}")
        return context_dict, val_context_dict

    def transform(self, context_dict, val_context_dict=None):
        return self._iterate_over_steps(context_dict, val_context_dict, training=False)

    def train(self, context_dict, val_context_dict=None):
        return self._iterate_over_steps(context_dict, val_context_dict, training=True)
