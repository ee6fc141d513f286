"""Import-level placeholders for the reference's experiments outside the hot path.

The reference's own entry scripts import names of experiments that SURVEY
§8(f)4 leaves out (the ClassificationHead baseline blend, NewAttention,
ReducingModel, the attention-weight / attention-reduce trainers, InfoNCE
datasets), e.g. ``scripts/eval.py:6-20`` imports ``ClassificationComponent``
even though the path it runs never constructs one.  Each such name exists here
so that ``from news_rec_utils.components import (...)`` resolves exactly as
against the reference; constructing or calling one raises ``OutOfScopeError``
naming the reference anchor.  None of them is implemented.
"""
from __future__ import annotations


class OutOfScopeError(NotImplementedError):
    """Raised when a placeholder of an out-of-scope reference experiment is used."""


def _message(name: str, anchor: str) -> str:
    return (f"{name} ({anchor}) is a reference experiment outside the MI355X hot path "
            "(SURVEY §8(f)4, DESIGN §7); only the name is provided so the reference's imports resolve")


def placeholder_class(name: str, anchor: str, module: str, base: type = object) -> type:
    """A class named ``name`` (in ``module``) whose construction raises OutOfScopeError."""
    msg = _message(name, anchor)

    def _raise(self, *args, **kwargs):
        raise OutOfScopeError(msg)

    body = {m: _raise for m in getattr(base, "__abstractmethods__", ())}  # so construction reaches __init__
    body.update({"__init__": _raise, "__doc__": msg, "__module__": module, "out_of_scope": True})
    return type(name, (base,), body)


def placeholder_function(name: str, anchor: str, module: str):
    """A function named ``name`` (in ``module``) whose call raises OutOfScopeError."""
    msg = _message(name, anchor)

    def fn(*args, **kwargs):
        raise OutOfScopeError(msg)

    fn.__name__ = fn.__qualname__ = name
    fn.__module__ = module
    fn.__doc__ = msg
    fn.out_of_scope = True
    return fn
