"""ctypes binding of librs_hip.so (the C-ABI declared in include/rs_capi.h).

``import torch`` happens first so that the process has exactly one HIP runtime
(torch's bundled libamdhip64.so.7, which the .so then binds to by SONAME).
There is no fallback: if the library is missing or a call fails, this module
raises.  Device tensors are passed as raw pointers; streams as
``torch.cuda.current_stream().cuda_stream``.
"""
from __future__ import annotations

import ctypes as C
import threading
from pathlib import Path

import torch  # noqa: F401  (loads the HIP runtime before the extension)

_LIB_PATH = Path(__file__).resolve().parent / "librs_hip.so"

P = C.c_void_p
I = C.c_int
L = C.c_int64
F = C.c_float
U64 = C.c_uint64

# name -> (restype, argtypes); must match include/rs_capi.h and include/rs_batchio.h
SIGNATURES = {
    "rs_version": (C.c_char_p, []),
    "rs_last_error_string": (C.c_char_p, []),
    "rs_set_option": (I, [I, I]),
    "rs_peer_state_bytes": (L, []),
    "rs_peer_mailbox_bytes": (L, [I, L]),
    "rs_peer_alloc": (I, [L, P]),
    "rs_peer_free": (I, [P]),
    "rs_peer_ipc_handle": (I, [P, P]),
    "rs_peer_ipc_open": (I, [P, P]),
    "rs_peer_ipc_close": (I, [P]),
    "rs_peer_a2a": (I, [P, L, P, I, I, P, I, L, P, P]),
    "rs_peer_gather_a2a": (I, [P, L, P, L, I, P, I, I, P, I, L, P, P]),
    "rs_get_option": (I, [I]),
    "rs_diag_empty": (I, [I, I, P]),
    "rs_diag_wave_slots": (I, [I, I, I, P, P]),
    "rs_diag_mfma_chain": (I, [I, I, I, I, P, P, P]),
    "rs_diag_icache": (I, [I, I, I, P, P, P]),
    "rs_embed_gather": (I, [P, I, L, P, L, I, P, P, P, I, I, P, L, L, P, P]),
    "rs_fm_prepared_size": (L, [I, I, I, I]),
    "rs_fm_prepare": (I, [P, P, I, I, I, I, P, P]),
    "rs_embed_fm_fwd": (I, [P, I, L, P, L, I, P, P, P, I, I, P, P, I, P, P, L, P, P]),
    "rs_embed_fm_fwd_hm": (I, [P, I, L, P, L, I, P, P, P, P, P, I, I, P, P, I, P, P, L, P, P]),
    "rs_embed_fm_fwd_hm_stream": (I, [P, I, L, L, P, L, L, I, P, P, P, I, I, P, P, I, P, L, L, I, L, I, P, P]),
    "rs_fm_fwd": (I, [P, L, I, P, P, I, P, L, P]),
    "rs_fm_onehot_fwd": (I, [P, I, L, P, L, I, P, P, I, P, P, P, I, P, L, P, P]),
    "rs_cross_prepared_size": (L, [I, I]),
    "rs_cross_prepare": (I, [P, P, I, I, P, P]),
    "rs_cross_fwd": (I, [P, L, I, I, P, P, L, L, P]),
    "rs_embed_cross_fwd": (I, [P, I, L, P, L, I, P, P, P, I, I, I, P, P, L, L, P, P]),
    "rs_embed_cross_fwd_hm": (I, [P, I, L, P, L, I, P, P, P, P, P, I, I, I, P, P, L, L, P, P]),
    "rs_dcn_fused_ok": (I, [I, I, I, I, I, P]),
    "rs_dcn_fwd": (I, [P, I, L, P, L, I, P, P, P, I, I, I, P, I, P, P, P, P, L, P, P]),
    "rs_dcn_fwd_hm": (I, [P, I, L, P, L, I, P, P, P, P, P, I, I, I, P, I, P, P, P, P, L, P, P]),
    "rs_inner_product_fwd": (I, [P, I, I, P, L, L, P]),
    "rs_embed_inner_fwd": (I, [P, I, L, P, P, P, I, I, P, L, L, P, P]),
    "rs_embed_inner_fwd_hm": (I, [P, I, L, P, P, P, P, P, I, I, P, L, L, P, P]),
    "rs_outer_prepared_size": (L, [I, I]),
    "rs_outer_prepare": (I, [P, I, I, P, P]),
    "rs_outer_product_fwd": (I, [P, I, I, P, P, L, L, P]),
    "rs_embed_product_fwd": (I, [P, I, L, P, P, P, I, I, I, P, P, L, L, P, P]),
    "rs_embed_product_fwd_hm": (I, [P, I, L, P, P, P, P, P, I, I, I, P, P, L, L, P, P]),
    "rs_din_attention_fwd": (I, [P, P, P, P, I, I, P, P, P, I, P, P, P, I, P, P, P, L, P]),
    "rs_din_attention_dice_fwd": (I, [P, P, P, P, I, I, I, P, P, P, F, P, P, P, L, P]),
    "rs_din_prepared_size": (L, [I, I, I, I]),
    "rs_din_prepare": (I, [P, P, P, I, P, P, P, I, P, P, I, I, P, P]),
    "rs_din_attention_ids_fwd": (I, [P, I, L, P, L, I, I, P, L, I, I, P, P, P, L, L, P, P]),
    "rs_din_attention_ids_cand_fwd": (I, [P, I, L, P, L, I, I, P, L, I, I, P, P, P, L, P, L, L, P, P]),
    "rs_din_forward_ids_supported": (I, [I, I, I, I, I, P]),
    "rs_din_forward_ids": (I, [P, I, L, P, L, I, I, P, L, I, I, P, P, L, P, P, I, P, P, P, P, L, I, P, P, P, P, P,
                               P, P, L, P, P]),
    "rs_dense_fwd": (I, [P, L, P, P, P, I, P, L, L, I, I, P]),
    "rs_dense_prelu_rows_fwd": (I, [P, L, P, P, P, I, P, L, L, I, I, P]),
    "rs_din_attention_gen_workspace_size": (L, [L, I, I, I, P]),
    "rs_din_attention_gen_fwd": (I, [P, P, P, P, I, I, I, P, P, P, P, P, P, P, L, P, L, P]),
    "rs_mlp_prepared_size": (L, [I, P]),
    "rs_mlp_prepare": (I, [I, P, P, P, P, P, P, P]),
    "rs_mlp_fwd": (I, [P, L, I, P, P, P, P, L, I, P, F, F, L, P]),
    "rs_mlp_affine_fwd": (I, [P, L, P, P, I, P, P, P, P, L, I, P, F, F, L, P]),
    "rs_mlp_affine_pieces_fwd": (I, [P, L, P, P, I, P, P, P, P, L, I, P, F, F, L, I, P, P, P, P, P, P, P, P, P]),
    "rs_concat_pieces": (I, [I, P, P, P, P, P, P, P, P, L, L, P, P]),
    "rs_deepfm_fused_ok": (I, [I, I, I, I, I, P]),
    "rs_deepfm_fwd": (I, [P, I, L, P, L, I, P, P, P, I, I, P, P, I, I, P, P, P, F, F, P, P, L, P, P]),
    "rs_deepfm_fwd_hm": (I, [P, I, L, P, L, I, P, P, P, P, P, I, I, P, P, I, I, P, P, P, F, F, P, P, L, P, P]),
    "rs_affine_act": (I, [P, L, P, P, P, I, P, L, L, I, P]),
    "rs_sigmoid_combine": (I, [P, P, F, F, P, L, P]),
    "rs_dice_fwd": (I, [P, L, P, P, F, P, P, L, L, I, P]),
    "rs_shard_workspace_size": (L, [L, I]),
    "rs_shard_bucketize": (I, [P, I, L, P, P, I, L, L, I, P, P, P, P, P, P]),
    "rs_shard_slot_bucketize": (I, [P, I, L, P, P, I, L, L, I, I, P, P, P, P, P, P, P]),
    "rs_gather_rows": (I, [P, L, I, P, L, P, P, P]),
    "rs_sort_pairs_workspace_size": (L, [L]),
    "rs_sort_pairs_u32": (I, [P, P, P, P, L, I, P, P]),
    "rs_inclusive_sum_workspace_size": (L, [L]),
    "rs_inclusive_sum_i32": (I, [P, P, L, P, P]),
    "rs_unpermute_rows": (I, [P, P, I, L, P, P]),
    "rs_rows_fm_fwd": (I, [P, P, L, I, I, I, P, P, I, P, L, P]),
    "rs_cb_write": (I, [C.c_char_p, L, I, I, I, P, P, P, P, P]),
    "rs_cb_open": (P, [C.c_char_p]),
    "rs_cb_info": (I, [P, P, P, P, P, P, P]),
    "rs_cb_read": (I, [P, L, L, P, P, P]),
    "rs_cb_close": (None, [P]),
    "rs_fm_train_workspace_size": (L, [L, I, I, I]),
    "rs_fm_train_step": (I, [P, I, L, P, L, I, P, P, I, I, P, P, P, L, P, L, F, F, F, P, P, P, P]),
    "rs_gemm_workspace_size": (L, [L, L, L]),
    "rs_gemm": (I, [I, I, L, L, L, F, P, L, P, L, F, P, L, P, L, P, L, P]),
    "rs_col_sum": (I, [P, L, L, L, P, P]),
    "rs_dropout": (I, [P, L, L, L, F, U64, U64, P]),
    "rs_dropout_at": (I, [P, L, L, L, F, U64, P, U64, P]),
    "rs_dropout_advance": (I, [P, U64, P]),
    "rs_sgd_update": (I, [P, P, L, F, F, P]),
    "rs_sgd_update_multi": (I, [I, P, P, P, P, F, P]),
    "rs_head_grad": (I, [P, P, P, L, F, F, P, P, P, P]),
    "rs_head_grad_scaled": (I, [P, P, P, L, F, F, F, P, P, P, P]),
    "rs_bce_prob_grad": (I, [P, L, P, L, P, P, P]),
    "rs_inner_product_bwd": (I, [P, L, P, L, P, L, I, I, L, P, L, P]),
    "rs_outer_product_bwd": (I, [P, L, P, L, P, I, I, L, P, L, P]),
    "rs_bi_interaction_bwd": (I, [P, L, P, L, I, I, L, P, L, P]),
    "rs_outer_product_w_grad": (I, [P, L, P, L, I, I, L, P, P]),
    "rs_din_att_concat": (I, [P, P, L, I, I, P, P]),
    "rs_din_att_concat_bwd": (I, [P, P, P, L, I, I, P, L, P, P]),
    "rs_prelu_rows_fwd": (I, [P, L, I, P, I, P, P]),
    "rs_prelu_rows_bwd_workspace_size": (L, [L, I, I]),
    "rs_prelu_rows_bwd": (I, [P, P, L, I, P, I, P, P, P, L, P]),
    "rs_din_att_prelu_fwd": (I, [P, P, P, P, P, P, P, P, P, L, I, I, I, I, P, P, P, P]),
    "rs_din_att_prelu_bwd_workspace_size": (L, [L, I, I, I, I]),
    "rs_din_att_prelu_bwd": (I, [P, P, P, P, P, P, P, P, P, L, I, I, I, I, P, P, P, P, P, P, P, P, P, P, L, P]),
    "rs_col_sum_workspace_size": (L, [L, L]),
    "rs_col_sum_split": (I, [P, L, L, L, P, P, L, P]),
    "rs_masked_softmax_pool": (I, [P, P, I, L, P, L, I, I, P, P, L, P]),
    "rs_masked_softmax_pool_bwd": (I, [P, P, I, L, P, P, L, L, I, I, P, P, P]),
    "rs_bn_train_fwd": (I, [P, L, L, I, P, P, F, F, P, P, P, P, P, L, P]),
    "rs_dice_train_workspace_size": (L, [L, I]),
    "rs_dice_train_fwd": (I, [P, L, I, P, F, F, P, P, P, P, P, P, L, P]),
    "rs_dice_train_bwd": (I, [P, L, I, P, P, P, F, P, P, P, P, L, P]),
    "rs_bn_train_bwd": (I, [P, L, L, I, P, P, P, F, P, L, P, L, P, P, P]),
    "rs_scatter_rows": (I, [P, L, I, I, P, L, P, P]),
    "rs_shard_dedup_workspace_size": (L, [L, I]),
    "rs_shard_dedup_route": (I, [P, I, L, P, P, I, L, L, I, L, P, P, P, P, P, P]),
    "rs_shard_dedup_grad": (I, [P, L, I, I, L, I, P, P, P, P]),
    "rs_fm_x_grad": (I, [P, L, P, P, P, L, I, I, P, P, L, P]),
    "rs_fm_param_grads": (I, [P, L, P, P, L, I, I, P, P, P, P, P]),
    "rs_fm_param_grads_strided": (I, [P, L, P, L, P, L, P, L, I, I, P, P, P, P]),
    "rs_shard_fm_combine_grad": (I, [P, L, I, L, P, L, I, I, I, P, P, I, P, F, P, P, L, P, P]),
    "rs_shard_owner_fm_grad": (I, [P, L, I, I, P, L, I, I, P, P, I, P, L, L, P, P, P, P, P]),
    "rs_cross_train_fwd": (I, [P, L, I, I, P, P, L, P, P, P, L, P]),
    "rs_cross_train_bwd": (I, [P, L, I, I, P, L, P, P, L, P, P, P, L, P]),
    "rs_embedding_sgd_workspace_size": (L, [L]),
    "rs_embedding_sgd": (I, [P, L, I, P, I, L, P, P, I, L, P, L, F, P, P, P]),
    "rs_embedding_sgd_strided": (I, [P, L, I, P, I, L, P, P, I, L, P, L, L, F, P, P, P]),
    "rs_ffm_train_fwd": (I, [P, I, L, P, L, I, P, P, P, P, P, I, I, P, L, P, P, P, P]),
    "rs_l2_decay": (I, [P, L, F, F, P]),
    "rs_fm_partial_width": (I, [I]),
    "rs_embed_pair_pool_fwd": (I, [P, I, L, P, P, P, I, I, I, P, L, I, P, L, I, P, P, I, P, L, P, P]),
    "rs_pair_products_fwd": (I, [P, L, I, I, L, P, P]),
    "rs_attention_pool_fwd": (I, [P, L, I, I, L, P, P]),
    "rs_ffm_fwd": (I, [P, I, L, P, L, I, P, P, P, P, P, I, I, I, P, L, P, P]),
    "rs_shard_field_route": (I, [P, I, L, P, P, I, L, L, I, P, I, L, P, P, P]),
    "rs_shard_row_route": (I, [P, I, L, P, P, I, L, L, I, P, I, P, P, P, P]),
    "rs_shard_owner_fm": (I, [P, L, I, I, P, L, I, I, I, P, I, P, L, L, P, P]),
    "rs_shard_fm_combine": (I, [P, L, I, L, P, L, I, I, I, P, P, I, P, P]),
    "rs_shard_fm_pipe": (I, [P, I, I, P, L, P, L, P, P, I, L, P, P, L, P, I, P, I, L, I, I, I, P, P, I, P, P]),
    "rs_shard_fm_pipe_peer": (I, [P, P, P, I, I, I, I, P, L, P, L, P, P, I, L, P, P, L, P, I, I, L, I, I, I, P, P, I,
                                  P, P, I, P, I, L, P, P]),
}

ID_I32, ID_I64, ID_F32 = 0, 1, 2
FLAG_BAD_ID, FLAG_LAYOUT, FLAG_TIMEOUT = 1, 2, 4  # rs_flag bits of the device error flag
_FLAG_NAMES = {FLAG_BAD_ID: "RS_FLAG_BAD_ID: an embedding id out of range",
               FLAG_LAYOUT: "RS_FLAG_LAYOUT: the table's field row ranges overlap or decrease",
               FLAG_TIMEOUT: "RS_FLAG_TIMEOUT: a bounded in-kernel wait gave up (kernel logic error; outputs invalid)"}


def flag_names(bits: int) -> str:
    """Human-readable list of the rs_flag bits set in `bits`."""
    names = [n for b, n in _FLAG_NAMES.items() if bits & b]
    unknown = bits & ~sum(_FLAG_NAMES)
    if unknown:
        names.append(f"unknown bits {unknown:#x}")
    return "; ".join(names)
OPT_EMBED_FM_KERNEL = 0  # rs_option
OPT_MLP_UNROLL = 1
OPT_DEEPFM_KERNEL = 2
OPT_DIN_KERNEL = 3
OPT_PEER_FENCES = 4
OPT_CROSS_KERNEL = 5
ACT = {None: 0, "linear": 0, "relu": 1, "prelu": 2, "sigmoid": 3}

_lock = threading.Lock()
_lib = None


class RSError(RuntimeError):
    pass


_ALLOW_MISSING = False  # scripts only: bind an older build that lacks newer entries


def lib():
    """Load (once) and return the bound library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not _LIB_PATH.exists():
                raise ImportError(
                    f"{_LIB_PATH} is missing: build the HIP extension first "
                    "(python -c 'import __graft_entry__ as g; g.build()')")
            h = C.CDLL(str(_LIB_PATH))
            for name, (res, args) in SIGNATURES.items():
                if _ALLOW_MISSING and not hasattr(h, name):
                    continue  # an older build under A/B (scripts/ab_options.py --lib)
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _lib = h
    return _lib


def library_path() -> Path:
    return _LIB_PATH


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().rs_last_error_string().decode()
        raise RSError(f"{what or 'librs_hip'} failed ({status}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RSError("librs_hip kernels need device (HIP) tensors; got a CPU tensor")
    return t.data_ptr()


def sgd_update_multi(updates, lr, st) -> None:
    """One rs_sgd_update_multi launch for [(w, grad, n, l2)] (w / grad device
    tensors or raw pointers; n elements; l2 the Keras l2 factor)."""
    if not updates:
        return
    cnt = len(updates)
    ws = (C.c_void_p * cnt)(*[u[0] if isinstance(u[0], int) else ptr(u[0]) for u in updates])
    gs = (C.c_void_p * cnt)(*[u[1] if isinstance(u[1], int) else ptr(u[1]) for u in updates])
    ns = (C.c_int64 * cnt)(*[int(u[2]) for u in updates])
    l2 = (C.c_float * cnt)(*[float(u[3]) for u in updates])
    call("rs_sgd_update_multi", cnt, ws, gs, ns, l2, float(lr), st)


def set_option(option: int, value: int) -> int:
    """rs_set_option: returns the previous value; raises on an unknown option."""
    prev = lib().rs_set_option(int(option), int(value))
    if prev < 0:
        raise RSError(lib().rs_last_error_string().decode())
    return prev


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def id_kind(t) -> int:
    if t.dtype == torch.int32:
        return ID_I32
    if t.dtype == torch.int64:
        return ID_I64
    if t.dtype == torch.float32:
        return ID_F32
    raise TypeError(f"unsupported sparse id dtype {t.dtype} (int32, int64 or float32)")
