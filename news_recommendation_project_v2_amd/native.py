"""ctypes binding of ``libnewsrec_host.so`` (include/newsrec_host.h): the native
behaviours parser behind ``data_utils.split_impressions_and_history``.

``split_behaviors`` returns the reference's output dict, or ``None`` when the
native parser declines the input (non-ASCII text, labels that are not
"<id>-<digits>", non-string rows): the caller then runs the Python
restatement, which reproduces the reference's behaviour (including its
exceptions) exactly.
"""
from __future__ import annotations

import ctypes
import os
from itertools import islice
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

LIB_PATH = Path(__file__).resolve().with_name("libnewsrec_host.so")
SOURCES = (Path(__file__).resolve().with_name("csrc") / "host" / "behaviors.cpp",
           Path(__file__).resolve().parent.parent / "include" / "newsrec_host.h")
_LIB = None
_p = ctypes.c_void_p


def load():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.is_file():
            return None
        from ._lib import source_hash
        lib = ctypes.CDLL(os.fspath(LIB_PATH))
        lib.nrh_build_hash.restype = ctypes.c_char_p
        want, got = source_hash(SOURCES), lib.nrh_build_hash().decode("ascii", "replace")
        if want is not None and got != want:
            raise RuntimeError(f"{LIB_PATH} was built from other sources (build hash {got}, tree {want}): "
                               "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")
        lib.nrh_split_behaviors.restype = ctypes.c_int
        lib.nrh_split_behaviors.argtypes = [_p, _p, _p, _p, _p, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(_p)]
        lib.nrh_split_sizes.restype = ctypes.c_int
        lib.nrh_split_sizes.argtypes = [_p, _p]
        lib.nrh_split_copy.restype = ctypes.c_int
        lib.nrh_split_copy.argtypes = [_p] * 8
        lib.nrh_split_free.restype = None
        lib.nrh_split_free.argtypes = [_p]
        lib.nrh_last_error.restype = ctypes.c_char_p
        _LIB = lib
    return _LIB


def _pack(rows: Sequence[str]):
    lens = np.fromiter(map(len, rows), dtype=np.int64, count=len(rows))
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return "".join(rows).encode("ascii"), off


def split_behaviors(impressions: Sequence[str], history: Sequence[Optional[str]]) -> Optional[dict]:
    lib = load()
    if lib is None:
        return None
    imps = list(impressions)
    hists = list(history)
    if not all(isinstance(x, str) for x in imps):
        return None
    skip = np.fromiter((not h for h in hists), dtype=np.uint8, count=len(hists))
    if not all(isinstance(h, str) for h, s in zip(hists, skip) if not s):
        return None  # e.g. NaN (truthy, no .split): let the restatement raise like the reference
    hrows = [h if not s else "" for h, s in zip(hists, skip)]
    try:
        ib, ioff = _pack(imps)
        hb, hoff = _pack(hrows)
    except UnicodeEncodeError:
        return None
    label_present = 1 if "-" in imps[0] else 0
    handle = _p()
    rc = lib.nrh_split_behaviors(ib, ioff.ctypes.data, hb, hoff.ctypes.data, skip.ctypes.data, len(imps),
                                 label_present, ctypes.byref(handle))
    if rc != 0:
        return None
    try:
        sizes = np.zeros(6, dtype=np.int64)
        lib.nrh_split_sizes(handle, sizes.ctypes.data)
        n_news, nbytes, C, H, n_hist, n_lab = (int(x) for x in sizes)
        news_b = ctypes.create_string_buffer(max(nbytes, 1))
        news_off = np.zeros(n_news + 1, dtype=np.int64)
        imp_idx = np.zeros(C, dtype=np.int32)
        imp_len = np.zeros(len(imps), dtype=np.int32)
        hist_idx = np.zeros(H, dtype=np.int32)
        hist_len = np.zeros(n_hist, dtype=np.int32)
        labels = np.zeros(n_lab, dtype=np.int8)
        lib.nrh_split_copy(handle, news_b, news_off.ctypes.data, imp_idx.ctypes.data, imp_len.ctypes.data,
                           hist_idx.ctypes.data, hist_len.ctypes.data, labels.ctypes.data if n_lab else None)
    finally:
        lib.nrh_split_free(handle)
    raw = news_b.raw[:nbytes].decode("ascii")
    news_list = [raw[news_off[i]:news_off[i + 1]] for i in range(n_news)]
    if label_present:
        it = iter(labels.tolist())  # Python ints, like the reference's int(x[1])
        tuples = [tuple(islice(it, n)) for n in imp_len.tolist()]
    else:
        tuples = []
    return {
        "news_list": np.array(news_list),
        "impression_rev_ind_array": np.stack([imp_idx, np.repeat(np.arange(len(imp_len), dtype=np.int32), imp_len)]),
        "impression_len_list": imp_len,
        "history_rev_ind_array": np.stack([hist_idx, np.repeat(np.arange(len(hist_len), dtype=np.int32), hist_len)]),
        "history_len_list": hist_len,
        "labels": np.array(tuples, dtype=object),
    }
