"""ctypes binding of ``libnewsrec_hip.so`` (C-ABI declared in include/newsrec.h).

The library is built in-tree by ``__graft_entry__.build()`` (or
``make -C news_recommendation_project_v2_amd/csrc``).  There is no CPU or
PyTorch fallback: if the library is missing or a call fails, a
``NewsRecHIPError`` is raised.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from pathlib import Path
from typing import Optional, Sequence

LIB_PATH = Path(__file__).resolve().with_name("libnewsrec_hip.so")
CSRC = Path(__file__).resolve().with_name("csrc")
INCLUDE = Path(__file__).resolve().parent.parent / "include"
# translation units of libnewsrec_hip.so, in link order (also the hash order)
HIP_SOURCES = ("capi.hip", "gemm.hip", "pool_score.hip", "rowops.hip", "rank.hip", "encoder.hip", "train.hip",
               "metrics.hip", "comm.hip", "latent_train.hip", "final_train.hip")


def hip_source_files() -> list:
    return [CSRC / s for s in HIP_SOURCES] + [CSRC / "nr_common.h", INCLUDE / "newsrec.h"]


def source_hash(files: Sequence[Path]) -> Optional[str]:
    """First 16 hex digits of sha256 over the files' bytes, concatenated in
    order (the Makefile computes the same with `cat ... | sha256sum`); None
    when a source is absent (a library shipped without its sources)."""
    h = hashlib.sha256()
    for f in files:
        if not Path(f).is_file():
            return None
        h.update(Path(f).read_bytes())
    return h.hexdigest()[:16]


def embedded_hash(lib_path: Path, tag: bytes = b"nr-build-hash:") -> Optional[str]:
    """The build hash a library carries (read from its bytes, without loading it)."""
    try:
        data = Path(lib_path).read_bytes()
    except OSError:
        return None
    i = data.find(tag)
    return data[i + len(tag):i + len(tag) + 16].decode("ascii", "replace") if i >= 0 else None

NR_OK = 0
NR_F32 = 0
NR_BF16 = 1
NR_F16 = 2
NR_POOL_FINAL = 0
NR_POOL_LATENT = 1
NR_POOL_MEAN = 2
NR_POOL_NONE = -1
NR_EPI_NONE = 0
NR_EPI_RELU = 1
NR_EPI_EXP = 2
NR_EPI_GEGLU = 3
NR_EPI_RESADD = 4
NR_EPI_GELU = 5
NR_EPI_RELU_DROPOUT = 6
NR_EPI_DRELU = 7
NR_EPI_SOFTMAX64 = 8
NR_EPI_SOFTMAX64_BWD = 9

_p = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_int64
_f = ctypes.c_float

# name -> (restype, argtypes); must match include/newsrec.h
SIGNATURES = {
    "nr_version": (_i, []),
    "nr_build_hash": (ctypes.c_char_p, []),
    "nr_init": (_i, [_i]),
    "nr_last_error": (ctypes.c_char_p, []),
    "nr_residency_flush": (_i, []),
    "nr_rccl_version": (_i, []),
    "nr_latent_train_workspace_bytes": (_l, [_i, _l, _l, _l]),
    "nr_latent_train_step": (_i, [_p, _p, _l, _p]),
    "nr_final_train_workspace_bytes": (_l, [_i, _l, _l, _l]),
    "nr_final_train_step": (_i, [_p, _p, _l, _p]),
    "nr_comm_unique_id": (_i, [_p]),
    "nr_comm_init": (_i, [_p, _p, _i, _i]),
    "nr_comm_init_timeout": (_i, [_p, _p, _i, _i, _l]),
    "nr_comm_destroy": (_i, [_p]),
    "nr_allgather": (_i, [_p, _p, _p, _l, _p]),
    "nr_is_device_pointer": (_i, [_p]),
    "nr_set_persistent_workgroups": (_i, [_i]),
    "nr_persistent_workgroups": (_i, []),
    "nr_set_gemm_half_tail": (_i, [_i]),
    "nr_gemm": (_i, [_i, _i, _i, _l, _l, _l, _p, _l, _p, _l, _p, _p, _l, _p, _l, _p]),
    "nr_gemm_relu_dropout": (_i, [_i, _i, _l, _l, _l, _p, _l, _p, _l, _p, _p, _l, ctypes.c_uint64, _f, _p]),
    "nr_gemm_drelu": (_i, [_i, _i, _l, _l, _l, _p, _l, _p, _l, _p, _l, _p, _l, _f, _p]),
    "nr_gemm_grouped": (_i, [_i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "nr_gemm_grouped_tn": (_i, [_i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "nr_layernorm": (_i, [_i, _i, _l, _l, _p, _l, _p, _p, _f, _p, _l, _p]),
    "nr_gather_layernorm": (_i, [_i, _l, _l, _p, _l, _p, _i, _p, _p, _f, _p, _l, _p]),
    "nr_softmax64": (_i, [_l, _l, _p, _l, _i, _p, _l, _p]),
    "nr_row_inv_norm": (_i, [_i, _l, _l, _p, _l, _f, _p, _p]),
    "nr_pool_score": (_i, [_i, _i, _l, _p, _l, _p, _l, _p, _p, _p, _p, _p, _l, _p, _p, _p]),
    "nr_score_users": (_i, [_i, _l, _p, _p, _p, _l, _p, _p, _p, _l, _p, _p]),
    "nr_splitk_fixup": (_i, [_i, _i, _l, _l, _i, _p, _p, _p, _l, _p, _l, _l, ctypes.c_uint64, _f, _f, _p]),
    "nr_dense_rank": (_i, [_p, _p, _l, _p, _p, _p]),
    "nr_impression_metrics": (_i, [_p, _p, _p, _l, _p, _p, _p, _p]),
    "nr_final_attn_workspace_bytes": (_l, [_i, _l]),
    "nr_final_attn_transform": (_i, [_i, _l, _p, _l, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _l, _p]),
    "nr_latent_workspace_bytes": (_l, [_i, _l]),
    "nr_latent_transform": (_i, [_i, _l, _p, _l, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _l, _p]),
    "nr_latent_transform_lnfold": (_i, [_i, _l, _p, _l, _p, _p, _p, _p, _p, _p, _p, _p, _p, _l, _p]),
    "nr_row_stats": (_i, [_i, _l, _l, _p, _l, _f, _p, _p]),
    "nr_embed_ln": (_i, [_i, _l, _p, _p, _p, _p, _p, _p, _p, _f, _p, _p]),
    "nr_attention_varlen": (_i, [_i, ctypes.c_int32, _l, _p, _p, _p, _p, _p]),
    "nr_gather_rows": (_i, [_i, _i, _l, _l, _p, _l, _p, _p, _l, _p]),
    "nr_transpose": (_i, [_i, _i, _l, _l, _p, _l, _p, _l, _p]),
    "nr_final_pool_fwd": (_i, [_i, _l, _p, _p, _l, _p, _p, _p]),
    "nr_final_pool_bwd": (_i, [_i, _l, _p, _l, _p, _l, _p, _p, _p, _p, _l, _p, _l, _p]),
    "nr_cosine_margin": (_i, [_l, _p, _p, _l, _p, _p, _f, _p, _p, _p, _p, _p]),
    "nr_scatter_add_rows": (_i, [_i, _l, _l, _p, _l, _p, _p, _l, _p]),
    "nr_col_sum": (_i, [_i, _l, _l, _p, _l, _p, _p]),
    "nr_ln_param_grad": (_i, [_i, _l, _l, _p, _l, _p, _f, _p, _l, _p, _p, _p]),
    "nr_sumsq": (_i, [_l, _p, _p, _p]),
    "nr_layernorm_bwd": (_i, [_l, _l, _p, _l, _p, _f, _p, _l, _p, _l, _p, _l, _p]),
    "nr_softmax64_bwd": (_i, [_i, _l, _l, _p, _l, _p, _l, _p, _l, _p]),
    "nr_geglu_fwd": (_i, [_i, _l, _l, _p, _l, _p, _l, _p]),
    "nr_geglu_bwd": (_i, [_i, _l, _l, _p, _l, _p, _l, _p, _l, _p]),
    "nr_adamw": (_i, [_l, _p, _p, _p, _p, _p, _l, _f, _f, _f, _f, _f, _f, _p, _p]),
    "nr_encoder_workspace_bytes": (_l, [_i, _l, _l]),
    "nr_encoder_forward": (_i, [_i, _i, _p, _p, _l, _p, _l, _p, _p, _p, _f, _l, _l, _p, _p, _i, _p, _p, _p, _p, _l,
                                _p]),
}


class EncoderLayer(ctypes.Structure):
    """struct nr_encoder_layer (include/newsrec.h): device pointers of one layer."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("wqkv", "bqkv", "wo", "bo", "ln1_g", "ln1_b", "w1", "b1", "w2", "b2",
                                             "ln2_g", "ln2_b")]


LATENT_TRAIN_PARAMS = ("tok_g", "tok_b", "latents", "nq_g", "nq_b", "nc_g", "nc_b", "Wq", "Wkv", "Wo", "nf_g", "nf_b",
                       "W1", "b1", "W2", "b2")
LATENT_TRAIN_GRADS = ("g_tok_g", "g_tok_b", "g_latents", "g_nq_g", "g_nq_b", "g_nc_g", "g_nc_b", "g_Wq", "g_Wkv",
                      "g_Wo", "g_nf_g", "g_nf_b", "g_W1", "g_b1", "g_W2", "g_b2")


class LatentTrainArgs(ctypes.Structure):
    """struct nr_latent_train_args (include/newsrec.h)."""
    _fields_ = ([("dtype", ctypes.c_int), ("tok_dtype", ctypes.c_int), ("B", ctypes.c_int64), ("U", ctypes.c_int64),
                 ("Hs", ctypes.c_int64)]
                + [(n, ctypes.c_void_p) for n in ("tok_last", "hist_idx", "hist_off", "pos", "neg")]
                + [("margin", ctypes.c_float)]
                + [(n, ctypes.c_void_p) for n in LATENT_TRAIN_PARAMS + LATENT_TRAIN_GRADS + ("loss", "users", "sumsq")])


FINAL_TRAIN_PARAMS = ("tok_g", "tok_b", "W1", "b1", "W2", "b2", "W3", "b3", "W4", "b4", "W5")
FINAL_TRAIN_GRADS = tuple("g_" + n for n in FINAL_TRAIN_PARAMS)


class FinalTrainArgs(ctypes.Structure):
    """struct nr_final_train_args (include/newsrec.h)."""
    _fields_ = ([("dtype", ctypes.c_int), ("tok_dtype", ctypes.c_int), ("B", ctypes.c_int64), ("U", ctypes.c_int64),
                 ("Hs", ctypes.c_int64)]
                + [(n, ctypes.c_void_p) for n in ("tok_last", "hist_idx", "hist_off", "pos", "neg")]
                + [("margin", ctypes.c_float), ("p", ctypes.c_float), ("seed", ctypes.c_uint64 * 3)]
                + [(n, ctypes.c_void_p) for n in FINAL_TRAIN_PARAMS + FINAL_TRAIN_GRADS + ("loss", "users", "sumsq")])


class NewsRecHIPError(RuntimeError):
    """A libnewsrec_hip call failed (or the library is not available)."""


_LIB = None


def load() -> ctypes.CDLL:
    """Load the HIP library once; raise loudly if it was not built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.is_file():
        raise NewsRecHIPError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the MI355X hot path)")
    lib = ctypes.CDLL(os.fspath(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    want = source_hash(hip_source_files())
    got = lib.nr_build_hash().decode("ascii", "replace")
    if want is not None and got != want:
        raise NewsRecHIPError(
            f"{LIB_PATH} was built from other sources (build hash {got}, tree {want}): rebuild it with "
            "`python -c 'import __graft_entry__ as g; g.build()'`")
    _LIB = lib
    return lib


def check(rc: int, name: str) -> None:
    if rc != NR_OK:
        msg = load().nr_last_error().decode(errors="replace")
        raise NewsRecHIPError(f"{name} failed ({rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def empty_cache() -> None:
    """torch.cuda.empty_cache() + nr_residency_flush(): the segments torch
    returns to the driver may be re-mapped later, so the library's cached
    "verified device range" tables are dropped with them (include/newsrec.h)."""
    import torch
    torch.cuda.empty_cache()
    if _LIB is not None:
        _LIB.nr_residency_flush()
