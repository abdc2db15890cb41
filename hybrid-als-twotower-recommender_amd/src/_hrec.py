"""ctypes binding of libhrec.so (the C-ABI declared in include/hrec.h).

Every wrapper takes torch tensors that already live on the current HIP
device and launches on torch's current stream; nothing here computes on the
host. If the library is missing the wrappers raise HrecError — there is no
CPU fallback on the product path.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HREC_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libhrec.so")

_c_i32 = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_u64 = ctypes.c_uint64
_c_dbl = ctypes.c_double
_c_sz = ctypes.c_size_t
_vp = ctypes.c_void_p

# name -> (restype, argtypes)
_SIGNATURES = {
    "hrec_abi_version": (_c_i32, []),
    "hrec_last_error": (ctypes.c_char_p, []),
    "hrec_synth_row_counts": (_c_i32, [_c_u64, _c_u64, _c_i64, _c_i64, _c_i64, _c_i32, _vp, _vp]),
    "hrec_synth_fill": (_c_i32, [_c_u64, _c_u64, _c_u64, _c_i64, _c_i64, _c_i64, _c_i32, _c_i32,
                                 _vp, _vp, _vp, _vp]),
    "hrec_scan_workspace_bytes": (_c_sz, [_c_i64]),
    "hrec_exclusive_scan_i64": (_c_i32, [_vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "hrec_encode_ids_workspace_bytes": (_c_sz, [_c_i64]),
    "hrec_encode_ids": (_c_i32, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_encode_ids_ex": (_c_i32, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_minmax_i64_workspace_bytes": (_c_sz, [_c_i64]),
    "hrec_minmax_i64": (_c_i32, [_vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "hrec_coo_to_csr_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "hrec_coo_to_csr": (_c_i32, [_vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_remap_i32": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _vp]),
    "hrec_rows_descending_pairs": (_c_i32, [_vp, _c_i64, _vp, _vp]),
    "hrec_coo_to_csr_sorted": (_c_i32, [_vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "hrec_als_init_factors": (_c_i32, [_c_u64, _c_i64, _c_i64, _c_i32, _c_i32, _vp, _vp]),
    "hrec_als_half_sweep_src64": (_c_i32, [_vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _c_dbl, _vp, _vp]),
    "hrec_f32_to_f64": (_c_i32, [_vp, _c_i64, _vp, _vp]),
    "hrec_als_half_sweep": (_c_i32, [_vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _c_dbl,
                                     _c_i32, _vp, _vp]),
    "hrec_transpose_f32": (_c_i32, [_vp, _c_i64, _c_i64, _vp, _c_i64, _vp]),
    "hrec_als_score": (_c_i32, [_vp, _vp, _c_i32, _vp, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _vp,
                                _vp]),
    "hrec_als_score_topk_workspace_bytes": (_c_sz, [_c_i32, _c_i64, _c_i32]),
    "hrec_als_score_topk": (_c_i32, [_vp, _vp, _c_i32, _vp, _c_i64, _c_i64, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp,
                                     _vp, _c_sz, _vp]),
    "hrec_als_items_bf16_bytes": (_c_sz, [_c_i64, _c_i32]),
    "hrec_als_items_bf16": (_c_i32, [_vp, _c_i64, _c_i64, _c_i32, _vp, _c_sz, _vp]),
    "hrec_als_score_topk_pruned_workspace_bytes": (_c_sz, [_c_i32, _c_i64, _c_i32, _c_i32]),
    "hrec_als_score_topk_pruned": (_c_i32, [_vp, _vp, _c_i32, _vp, _c_i64, _vp, _c_i64, _vp, _c_i64, _c_i32,
                                            _c_i32, _c_i32, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_als_score_topk_pruned_counts": (_c_i32, [_vp, _c_i32, _c_i64, _c_i32, _c_i32, _vp, _vp]),
    "hrec_topk_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_i32, _c_i32]),
    "hrec_topk_f32": (_c_i32, [_vp, _c_i64, _c_i64, _c_i64, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_topk_f64": (_c_i32, [_vp, _c_i64, _c_i64, _c_i64, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_cosine_sim": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _c_i64, _vp, _vp]),
    "hrec_cold_fallback_workspace_bytes": (_c_sz, [_c_i64, _c_i32]),
    "hrec_cold_fallback": (_c_i32, [_vp, _vp, _c_i64, _c_i32, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_rows_minmax_f32": (_c_i32, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp]),
    "hrec_fuse_rows_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_i32]),
    "hrec_fuse_rows_topk": (_c_i32, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i32, _c_i32, _c_i64, _vp, _vp,
                                     _vp, _c_sz, _vp]),
    "hrec_topk_f64_keyed": (_c_i32, [_vp, _vp, _c_i64, _c_i64, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_fuse_workspace_bytes": (_c_sz, [_c_i64, _c_i32]),
    "hrec_fuse_topk": (_c_i32, [_vp, _vp, _c_i32, _c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp,
                                _c_sz, _vp]),
}



class TTParams(ctypes.Structure):
    """hrec_tt_params (include/hrec.h)."""
    _fields_ = [("d", ctypes.c_int32), ("reserved", ctypes.c_int32)] + [
        (name, _vp) for name in ("user_emb", "item_emb", "man_emb", "cat_emb", "w1", "b1", "w2", "b2",
                                 "ln_user_gamma", "ln_user_beta", "ln_item_gamma", "ln_item_beta")]


class SparseTable(ctypes.Structure):
    """hrec_sparse_table (include/hrec.h)."""
    _fields_ = [("var", _vp), ("m", _vp), ("v", _vp), ("n_rows", ctypes.c_int64), ("dim", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("indices", _vp), ("grad_rows", _vp), ("mark", _vp), ("gsum", _vp)]


MAX_SPARSE_TABLES = 8
_PP = ctypes.POINTER(TTParams)
_SIGNATURES.update({
    "hrec_tt_item_forward": (_c_i32, [_PP, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp]),
    "hrec_tt_user_forward": (_c_i32, [_PP, _vp, _c_i64, _vp, _vp]),
    "hrec_tt_score": (_c_i32, [_vp, _c_i32, _vp, _c_i64, _c_i32, _vp, _vp]),
    "hrec_tt_pair_score": (_c_i32, [_vp, _vp, _c_i64, _c_i32, _vp, _vp]),
    "hrec_tt_item_inputs_workspace_bytes": (_c_sz, [_c_i64]),
    "hrec_tt_item_inputs": (_c_i32, [_vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_tt_train_workspace_bytes": (_c_sz, [_c_i32, _c_i64]),
    "hrec_tt_grad_len": (_c_sz, [_c_i32]),
    "hrec_tt_forward_backward": (_c_i32, [_PP, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _c_sz, _vp]),
    "hrec_adam_dense": (_c_i32, [_vp, _vp, _vp, _vp, _c_i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                 ctypes.c_float, _vp]),
    "hrec_f32_to_bf16": (_c_i32, [_vp, _c_i64, _vp, _vp]),
    "hrec_dot_scores": (_c_i32, [_vp, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _vp, _c_i64, _vp]),
    "hrec_dot_topk_workspace_bytes": (_c_sz, [_c_i32, _c_i64, _c_i32]),
    "hrec_dot_topk": (_c_i32, [_vp, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _c_i32, _vp, _c_i64, _vp, _vp, _vp, _vp,
                               _c_sz, _vp]),
    "hrec_dot_filter": (_c_i32, [_vp, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _vp, _c_i32, _c_i64, _c_i32, _vp, _vp,
                                 _vp, _vp]),
    "hrec_hybrid_scores_workspace_bytes": (_c_sz, [_c_i32, _c_i64]),
    "hrec_hybrid_scores": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _c_i64, _c_i32,
                                    _vp, _vp, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_hybrid_prune_workspace_bytes": (_c_sz, [_c_i32, _c_i64, _c_i32, _c_i32]),
    "hrec_hybrid_prune_minmax": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp,
                                          _c_i64, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_hybrid_prune_topk": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp,
                                        _c_i64, _c_i32, _vp, _vp, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_hybrid_prune_local": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp,
                                         _c_i64, _c_i32, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_sz,
                                         _vp]),
    "hrec_hybrid_prune_fallback_taken": (_c_i32, [_vp, _c_i32, _c_i64, _c_i32, _c_i32, _vp, _vp]),
    "hrec_hybrid_prune_survivors": (_c_i32, [_vp, _c_i32, _c_i64, _c_i32, _c_i32, _vp, _vp]),
    "hrec_comm_get_unique_id": (_c_i32, [_vp]),
    "hrec_comm_init": (_c_i32, [_c_i32, _c_i32, _vp, ctypes.POINTER(_vp)]),
    "hrec_comm_destroy": (_c_i32, [_vp]),
    "hrec_allgather": (_c_i32, [_vp, _vp, _vp, _c_sz, _c_i32, _vp]),
    "hrec_allreduce_minmax": (_c_i32, [_vp, _vp, _c_i32, _c_i64, _vp]),
    "hrec_adam_sparse": (_c_i32, [_vp, _vp, _vp, _c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp] +
                         [ctypes.c_float] * 6 + [_vp]),
    "hrec_adam_sparse_tables": (_c_i32, [ctypes.POINTER(SparseTable), _c_i32] + [ctypes.c_float] * 6 + [_vp]),
    "hrec_adam_sparse_tables_phase": (_c_i32, [ctypes.POINTER(SparseTable), _c_i32, _c_i32] + [ctypes.c_float] * 6
                                      + [_vp]),
})

class HybridBatch(ctypes.Structure):
    """hrec_hybrid_batch (include/hrec.h)."""
    _fields_ = [("als_users", _vp), ("als_rows", _vp), ("tt_users", _vp), ("als_items_t", _vp), ("tt_items", _vp),
                ("tt_items_t", _vp), ("prepared", _vp), ("als_ld", _c_i64), ("n_als_rows", _c_i64),
                ("tt_ld", _c_i64), ("als_items_ld", _c_i64), ("tt_items_ld", _c_i64), ("tt_items_t_ld", _c_i64),
                ("n_items", _c_i64), ("als_width", _c_i32), ("tt_width", _c_i32), ("n_users", _c_i32),
                ("dk", _c_i32)]


_HBP = ctypes.POINTER(HybridBatch)
_SIGNATURES.update({
    "hrec_hybrid_exact_items_bytes": (_c_sz, [_c_i64, _c_i32]),
    "hrec_hybrid_exact_prepare": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _c_i64, _c_i32, _c_i64, _c_i32, _vp, _vp]),
    "hrec_hybrid_exact_workspace_bytes": (_c_sz, [_c_i32, _c_i64, _c_i32]),
    "hrec_hybrid_exact_minmax": (_c_i32, [_HBP, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_hybrid_exact_topk": (_c_i32, [_HBP, _vp, _vp, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_hybrid_exact_local": (_c_i32, [_HBP, _c_i32, _c_i32, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "hrec_hybrid_exact_counts": (_c_i32, [_vp, _c_i32, _c_i64, _c_i32, _vp, _vp]),
})

ABI_VERSION = 7
_LIB = None


class HrecError(RuntimeError):
    """A libhrec call failed (or the library is not built)."""


def lib():
    """Load libhrec.so once. torch is imported first so the library binds to
    the HIP runtime torch already loaded (same soname libamdhip64.so.7)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise HrecError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " (no CPU fallback exists for the HIP hot path)")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.hrec_abi_version() != ABI_VERSION:
            raise HrecError("libhrec ABI version mismatch; rebuild the library")
        _LIB = handle
    return _LIB


def exported_symbols():
    return list(_SIGNATURES)


def _check(name, rc):
    if rc != 0:
        msg = lib().hrec_last_error().decode(errors="replace")
        raise HrecError(f"{name} failed ({rc}): {msg}")


def _stream():
    return _vp(torch.cuda.current_stream().cuda_stream)


def _dev(t, dtype, name):
    if t is None:
        return None
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise HrecError(f"{name}: expected a device tensor")
    if t.dtype != dtype:
        raise HrecError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise HrecError(f"{name}: tensor must be contiguous")
    return _vp(t.data_ptr())


def require_device():
    if not torch.cuda.is_available():
        raise HrecError("no HIP device visible: the MI355X hot path needs a GPU")


# ------------------------------------------------------------------ synth
def synth_row_counts(seed, threshold, row_begin, n_rows, n_cols, transposed, counts):
    _check("hrec_synth_row_counts", lib().hrec_synth_row_counts(
        seed, threshold, row_begin, n_rows, n_cols, int(transposed),
        _dev(counts, torch.int64, "counts"), _stream()))


def synth_fill(seed, seed2, threshold, row_begin, n_rows, n_cols, transposed, n_levels, indptr,
               indices, values):
    _check("hrec_synth_fill", lib().hrec_synth_fill(
        seed, seed2, threshold, row_begin, n_rows, n_cols, int(transposed), n_levels,
        _dev(indptr, torch.int64, "indptr"), _dev(indices, torch.int32, "indices"),
        _dev(values, torch.float32, "values"), _stream()))


def exclusive_scan(counts):
    """indptr[n+1] from counts[n] on the device."""
    n = counts.numel()
    out = torch.empty(n + 1, dtype=torch.int64, device=counts.device)
    ws_bytes = int(lib().hrec_scan_workspace_bytes(n))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=counts.device)
    _check("hrec_exclusive_scan_i64", lib().hrec_exclusive_scan_i64(
        _dev(counts, torch.int64, "counts"), n, _dev(out, torch.int64, "out"),
        _dev(ws, torch.uint8, "ws"), ws.numel(), _stream()))
    return out


# ----------------------------------------------------------------- ingest
def minmax_i64(x):
    """(min, max) of a non-empty int64 device tensor (host ints)."""
    n = x.numel()
    out = torch.empty(2, dtype=torch.int64, device=x.device)
    ws = torch.empty(max(int(lib().hrec_minmax_i64_workspace_bytes(n)), 16), dtype=torch.uint8, device=x.device)
    _check("hrec_minmax_i64", lib().hrec_minmax_i64(
        _dev(x, torch.int64, "x"), n, _dev(out, torch.int64, "out"), _dev(ws, torch.uint8, "ws"), ws.numel(),
        _stream()))
    lo, hi = out.tolist()
    return lo, hi


def encode_ids(ids, id_range=None, order=False):
    """numpy.unique(ids, return_inverse=True) on the device: ids int64[n] ->
    (sorted distinct ids int64[m], codes int32[n]). id_range = (lo, hi) with
    lo <= ids <= hi if known; else it is measured on the device first.
    order=True appends whether ids (hence codes) are non-decreasing and, when
    they are, the row pointer of rows = codes (int64[m + 1]; else None) — both
    read by the marking / code passes (hrec_encode_ids_ex), for coo_to_csr's
    rows_in_order / indptr."""
    n = ids.numel()
    dev = ids.device
    uniq = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    codes = torch.empty(n, dtype=torch.int32, device=dev)
    n_uniq = torch.zeros(1, dtype=torch.int64, device=dev)
    if n == 0:
        return (uniq[:0], codes, True, torch.zeros(1, dtype=torch.int64, device=dev)) if order else (uniq[:0], codes)
    lo, hi = minmax_i64(ids) if id_range is None else (int(id_range[0]), int(id_range[1]))
    ws = torch.empty(max(int(lib().hrec_encode_ids_workspace_bytes(n)), 16), dtype=torch.uint8, device=dev)
    desc = starts = None
    if order:
        desc = torch.zeros(1, dtype=torch.int32, device=dev)
        starts = torch.empty(min(n, hi - lo + 1) + 1, dtype=torch.int64, device=dev)
    _check("hrec_encode_ids_ex", lib().hrec_encode_ids_ex(
        _dev(ids, torch.int64, "ids"), n, lo, hi, _dev(uniq, torch.int64, "uniq"),
        _dev(n_uniq, torch.int64, "n_uniq"), _dev(codes, torch.int32, "codes"),
        _dev(desc, torch.int32, "descending") if order else None,
        _dev(starts, torch.int64, "starts") if order else None, _dev(ws, torch.uint8, "ws"),
        ws.numel(), _stream()))
    if order:
        m, d = torch.cat([n_uniq, desc.to(torch.int64)]).tolist()  # one host read
        return uniq[:m], codes, d == 0, (starts[: m + 1] if d == 0 else None)
    return uniq[: int(n_uniq.item())], codes


def coo_to_csr(rows, cols, vals, n_rows, alias=False, rows_in_order=None, indptr=None):
    """(indptr int64[n_rows+1], indices int32[nnz], values f32[nnz]) of the COO
    (rows, cols, vals), rows ascending, a row's entries in input order.
    alias=True: when rows are already in order the returned indices / values
    ARE cols / vals (no copy) — for callers that do not modify either after.
    rows_in_order: whether rows is non-decreasing, when the caller knows it
    (encode_ids(..., order=True)); None checks on the device. indptr: the
    row pointer encode_ids(..., order=True) returned for rows in order (with
    alias=True nothing runs on the device)."""
    nnz = rows.numel()
    dev = rows.device
    if cols.numel() != nnz or vals.numel() != nnz:
        raise HrecError("coo_to_csr: rows, cols and vals must have the same length")
    if indptr is not None and rows_in_order and alias:
        if indptr.numel() > n_rows + 1:
            raise HrecError("coo_to_csr: indptr has more than n_rows + 1 entries")
        if indptr.numel() < n_rows + 1:  # rows past the last code: empty (they end at nnz)
            indptr = torch.cat([indptr, torch.full((n_rows + 1 - indptr.numel(),), nnz, dtype=torch.int64,
                                                   device=dev)])
        return indptr, cols, vals
    indptr = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
    # rows already in order (e.g. ratings grouped by user): no sort needed
    if rows_in_order is None:
        flag = torch.empty(1, dtype=torch.int32, device=dev)
        _check("hrec_rows_descending_pairs", lib().hrec_rows_descending_pairs(
            _dev(rows, torch.int32, "rows"), nnz, _dev(flag, torch.int32, "out"), _stream()))
        in_order = int(flag.item()) == 0
    else:
        in_order = bool(rows_in_order)
    if in_order and alias:
        indices, values = cols, vals
    else:
        indices = torch.empty(nnz, dtype=torch.int32, device=dev)
        values = torch.empty(nnz, dtype=torch.float32, device=dev)
    if in_order:
        _check("hrec_coo_to_csr_sorted", lib().hrec_coo_to_csr_sorted(
            _dev(rows, torch.int32, "rows"), _dev(cols, torch.int32, "cols"), _dev(vals, torch.float32, "vals"),
            nnz, n_rows, _dev(indptr, torch.int64, "indptr"), _dev(indices, torch.int32, "indices"),
            _dev(values, torch.float32, "values"), _stream()))
        return indptr, indices, values
    ws = torch.empty(max(int(lib().hrec_coo_to_csr_workspace_bytes(nnz, n_rows)), 16), dtype=torch.uint8,
                     device=dev)
    _check("hrec_coo_to_csr", lib().hrec_coo_to_csr(
        _dev(rows, torch.int32, "rows"), _dev(cols, torch.int32, "cols"), _dev(vals, torch.float32, "vals"),
        nnz, n_rows, _dev(indptr, torch.int64, "indptr"), _dev(indices, torch.int32, "indices"),
        _dev(values, torch.float32, "values"), _dev(ws, torch.uint8, "ws"), ws.numel(), _stream()))
    return indptr, indices, values


def remap_i32(x, table):
    """x[i] = table[x[i]] in place on the device (ids outside the table -> -1)."""
    _check("hrec_remap_i32", lib().hrec_remap_i32(
        _dev(x, torch.int32, "x"), x.numel(), _dev(table, torch.int32, "table"), table.numel(), _stream()))
    return x


# -------------------------------------------------------------------- ALS
def als_init_factors(seed, row_begin, n_rows, k, kp, out):
    _check("hrec_als_init_factors", lib().hrec_als_init_factors(
        seed, row_begin, n_rows, k, kp, _dev(out, torch.float32, "out"), _stream()))


def als_half_sweep(indptr, indices, values, src_factors, k, reg_param, dst_factors, accum_mode=0, src64=None):
    """K1. src64 (optional): the source factors already converted to f64
    (f32_to_f64 of src_factors) — same results, no conversion per gathered
    row (hrec_als_half_sweep_src64; kp 64, accum_mode 0)."""
    n_rows = indptr.numel() - 1
    kp = dst_factors.shape[1]
    if src_factors.shape[1] != kp or dst_factors.shape[0] < n_rows:
        raise HrecError("als_half_sweep: factor shapes do not match")
    if src64 is not None:
        if accum_mode != 0 or src64.shape != src_factors.shape:
            raise HrecError("als_half_sweep: src64 needs accum_mode 0 and the source factors' shape")
        _check("hrec_als_half_sweep_src64", lib().hrec_als_half_sweep_src64(
            _dev(indptr, torch.int64, "indptr"), _dev(indices, torch.int32, "indices"),
            _dev(values, torch.float32, "values"), n_rows, _dev(src64, torch.float64, "src64"),
            src64.shape[0], k, kp, float(reg_param), _dev(dst_factors, torch.float32, "dst_factors"), _stream()))
        return
    _check("hrec_als_half_sweep", lib().hrec_als_half_sweep(
        _dev(indptr, torch.int64, "indptr"), _dev(indices, torch.int32, "indices"),
        _dev(values, torch.float32, "values"), n_rows,
        _dev(src_factors, torch.float32, "src_factors"), src_factors.shape[0], k, kp,
        float(reg_param), int(accum_mode), _dev(dst_factors, torch.float32, "dst_factors"),
        _stream()))


def f32_to_f64(x, out=None):
    """Exact f32 -> f64 copy on the device (hrec_f32_to_f64)."""
    x = x.contiguous()
    if out is None:
        out = torch.empty(x.shape, dtype=torch.float64, device=x.device)
    if out.numel() != x.numel():
        raise HrecError("f32_to_f64: size mismatch")
    _check("hrec_f32_to_f64", lib().hrec_f32_to_f64(_dev(x, torch.float32, "in"), x.numel(),
                                                    _dev(out, torch.float64, "out"), _stream()))
    return out


def transpose(x, pad=4):
    """[rows, cols] -> [cols, ld] with ld = rows rounded up to `pad` (the
    padding columns are zero) so vector loads along rows stay aligned."""
    rows, cols = x.shape
    ld = -(-rows // pad) * pad
    out = torch.zeros((cols, ld), dtype=torch.float32, device=x.device)
    _check("hrec_transpose_f32", lib().hrec_transpose_f32(
        _dev(x, torch.float32, "in"), rows, cols, _dev(out, torch.float32, "out"), ld, _stream()))
    return out


def als_score(user_factors, user_rows, item_factors_t, item_rows, n_items, k, out=None):
    kp = user_factors.shape[1]
    n_users = user_rows.numel()
    if out is None:
        out = torch.empty((n_users, n_items), dtype=torch.float32, device=user_factors.device)
    _check("hrec_als_score", lib().hrec_als_score(
        _dev(user_factors, torch.float32, "user_factors"), _dev(user_rows, torch.int64, "user_rows"),
        n_users, _dev(item_factors_t, torch.float32, "item_factors_t"), item_factors_t.shape[1],
        _dev(item_rows, torch.int64, "item_rows"), n_items, k, kp,
        _dev(out, torch.float32, "out"), _stream()))
    return out


def als_score_topk(user_factors, user_rows, item_factors_t, n_items, k, top_k, check_overflow=True,
                   overflow_out=None):
    """Top-k of the JVM-exact ALS scores over items [0, n_items) for each
    (known) user, without materialising the score matrix. Falls back to the
    full score matrix + top-k when a user's survivor list overflowed.
    overflow_out (device int32 [1], optional) receives the library's overflow
    flag (with check_overflow=False the caller resolves it later)."""
    kp = user_factors.shape[1]
    B = user_rows.numel()
    kk = min(int(top_k), int(n_items))
    dev = user_factors.device
    out_i = torch.empty((B, kk), dtype=torch.int64, device=dev)
    out_v = torch.empty((B, kk), dtype=torch.float32, device=dev)
    # zeroed by the library on the stream
    flag = overflow_out if overflow_out is not None else torch.empty(1, dtype=torch.int32, device=dev)
    need = int(lib().hrec_als_score_topk_workspace_bytes(B, n_items, kk))
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _check("hrec_als_score_topk", lib().hrec_als_score_topk(
        _dev(user_factors, torch.float32, "user_factors"), _dev(user_rows, torch.int64, "user_rows"), B,
        _dev(item_factors_t, torch.float32, "item_factors_t"), item_factors_t.shape[1], n_items, k, kp, kk,
        _dev(out_i, torch.int64, "out_idx"), _dev(out_v, torch.float32, "out_val"),
        _dev(flag, torch.int32, "overflow"), _dev(ws, torch.uint8, "ws"), need, _stream()))
    if check_overflow and int(flag.item()) != 0:
        scores = als_score(user_factors, user_rows, item_factors_t, None, n_items, k)
        return topk(scores, kk)
    return out_i, out_v


def als_items_bf16(item_factors, k):
    """The pruned ALS top-k's item operand (hrec_als_items_bf16): bf16 rows
    [N][dk] + the largest row norm, one uint8 device buffer (once per item
    matrix; item_factors row-major f32 [N, >= k])."""
    n = int(item_factors.shape[0])
    need = int(lib().hrec_als_items_bf16_bytes(n, int(k)))
    out = torch.empty(need, dtype=torch.uint8, device=item_factors.device)
    _check("hrec_als_items_bf16", lib().hrec_als_items_bf16(
        _dev(item_factors, torch.float32, "item_factors"), item_factors.stride(0), n, int(k),
        _vp(out.data_ptr()), need, _stream()))
    return out


def als_score_topk_pruned(user_factors, user_rows, item_factors_t, item_factors, items_bf16, n_items, k, top_k,
                          check_overflow=True, overflow_out=None, workspace=None):
    """als_score_topk with the bf16 matrix-core bound in front of the exact
    chain (hrec_als_score_topk_pruned): the same (ids, scores). item_factors
    is the row-major copy of item_factors_t, items_bf16 from als_items_bf16.
    workspace (uint8 device, optional) is reused when large enough. For
    top_k <= 8 an overflow is resolved on the device inside the call (no
    host read); above, the overflow flag falls back to the full score matrix
    + top-k as als_score_topk does (check_overflow)."""
    kp = user_factors.shape[1]
    B = user_rows.numel()
    kk = min(int(top_k), int(n_items))
    dev = user_factors.device
    if item_factors.stride(1) != 1 or item_factors.shape[0] < n_items:
        raise HrecError("als_score_topk_pruned: item_factors must be row-major with >= n_items rows")
    out_i = torch.empty((B, kk), dtype=torch.int64, device=dev)
    out_v = torch.empty((B, kk), dtype=torch.float32, device=dev)
    flag = overflow_out if overflow_out is not None else torch.empty(1, dtype=torch.int32, device=dev)
    need = int(lib().hrec_als_score_topk_pruned_workspace_bytes(B, n_items, kk, int(k)))
    ws = workspace if workspace is not None and workspace.numel() >= need else \
        torch.empty(need, dtype=torch.uint8, device=dev)
    _check("hrec_als_score_topk_pruned", lib().hrec_als_score_topk_pruned(
        _dev(user_factors, torch.float32, "user_factors"), _dev(user_rows, torch.int64, "user_rows"), B,
        _dev(item_factors_t, torch.float32, "item_factors_t"), item_factors_t.shape[1],
        _dev(item_factors, torch.float32, "item_factors"), item_factors.stride(0),
        _dev(items_bf16, torch.uint8, "items_bf16"), n_items, int(k), kp, kk,
        _dev(out_i, torch.int64, "out_idx"), _dev(out_v, torch.float32, "out_val"),
        _dev(flag, torch.int32, "overflow"), _dev(ws, torch.uint8, "ws"), ws.numel(), _stream()))
    if check_overflow and kk > 8 and int(flag.item()) != 0:
        scores = als_score(user_factors, user_rows, item_factors_t, None, n_items, k)
        return topk(scores, kk)
    return out_i, out_v


def als_topk_pruned_counts(ws, B, n_items, top_k, k):
    """Diagnostics of the last als_score_topk_pruned call on workspace ws:
    (pairs the bf16 bound kept per user, candidates per user), int32 [B]
    each (hrec_als_score_topk_pruned_counts)."""
    out = torch.zeros(2 * B, dtype=torch.int32, device=ws.device)
    _check("hrec_als_score_topk_pruned_counts", lib().hrec_als_score_topk_pruned_counts(
        _dev(ws, torch.uint8, "ws"), int(B), int(n_items), int(top_k), int(k), _dev(out, torch.int32, "out"),
        _stream()))
    return out[:B].clone(), out[B:].clone()


# ------------------------------------------------------------------ top-k
def topk(vals, top_k):
    """Stable descending top-k of each row of a 2-D f32/f64 device tensor."""
    if vals.dim() == 1:
        vals = vals.unsqueeze(0)
    n_rows, n = vals.shape
    kk = min(int(top_k), n)
    dev = vals.device
    is64 = vals.dtype == torch.float64
    out_i = torch.empty((n_rows, kk), dtype=torch.int64, device=dev)
    out_v = torch.empty((n_rows, kk), dtype=vals.dtype, device=dev)
    if kk == 0:
        return out_i, out_v
    ws_bytes = int(lib().hrec_topk_workspace_bytes(n_rows, n, kk, int(is64)))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    fn = lib().hrec_topk_f64 if is64 else lib().hrec_topk_f32
    _check("hrec_topk", fn(_dev(vals, vals.dtype, "vals"), n_rows, n, vals.stride(0), kk,
                           _dev(out_i, torch.int64, "out_idx"), _dev(out_v, vals.dtype, "out_val"),
                           _dev(ws, torch.uint8, "ws"), ws_bytes, _stream()))
    return out_i, out_v


# ----------------------------------------------------------------- fusion
def fuse_topk(als, tt, als_wins, top_k, want_fused=True, minmax=None):
    """als: f64 [n]; tt: f32 or f64 [n] (device). Returns (idx, score, fused).
    minmax (optional f64 [4] device tensor) receives (als min, als max, tt min, tt max)."""
    n = als.numel()
    dev = als.device
    tt_f32 = tt.dtype == torch.float32
    kk = min(int(top_k), n)
    out_i = torch.empty(max(kk, 1), dtype=torch.int64, device=dev)
    out_s = torch.empty(max(kk, 1), dtype=torch.float64, device=dev)
    fused = torch.empty(n, dtype=torch.float64, device=dev) if want_fused else None
    ws_bytes = int(lib().hrec_fuse_workspace_bytes(n, kk))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    _check("hrec_fuse_topk", lib().hrec_fuse_topk(
        _dev(als, torch.float64, "als"), _dev(tt, tt.dtype, "tt"), int(tt_f32), n, int(bool(als_wins)),
        kk, _dev(out_i, torch.int64, "out_idx"), _dev(out_s, torch.float64, "out_score"),
        _dev(fused, torch.float64, "out_fused"), _dev(minmax, torch.float64, "out_minmax"),
        _dev(ws, torch.uint8, "ws"), ws_bytes, _stream()))
    return out_i[:kk], out_s[:kk], fused


# ------------------------------------------------------------ cold start
def cosine_sim(feats, query_rows):
    """[n_query, n_items] f64 cosine similarities (self = -inf)."""
    n_items, dim = feats.shape
    out = torch.empty((query_rows.numel(), n_items), dtype=torch.float64, device=feats.device)
    _check("hrec_cosine_sim", lib().hrec_cosine_sim(
        _dev(feats, torch.float64, "feats"), n_items, dim, _dev(query_rows, torch.int64, "query_rows"),
        query_rows.numel(), _dev(out, torch.float64, "out"), _stream()))
    return out


COLD_MAX_DIM = 16  # hrec_cold_fallback's feature width limit


def cold_fallback(feats, ratings, want_idx=False):
    """The cold-start fallback of every item at once (hrec_cold_fallback,
    src/als_model.py:78-86,93-104): feats [n, dim] f64 (dim <= 16), ratings
    [n] f64 (the items' 'rating'), both device. Returns (mean f64 [n]: the
    mean rating of the <= 3 most similar other items with cosine > 0.5, 0
    where there is none; count int32 [n]; idx int32 [n, 3] of those items'
    rows, -1 padded, when want_idx)."""
    n, dim = feats.shape
    dev = feats.device
    mean = torch.empty(n, dtype=torch.float64, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    idx = torch.empty((n, 3), dtype=torch.int32, device=dev) if want_idx else None
    need = int(lib().hrec_cold_fallback_workspace_bytes(n, dim))
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _check("hrec_cold_fallback", lib().hrec_cold_fallback(
        _dev(feats, torch.float64, "feats"), _dev(ratings, torch.float64, "ratings"), n, dim,
        _dev(mean, torch.float64, "out_mean"), _dev(cnt, torch.int32, "out_count"),
        _dev(idx, torch.int32, "out_idx") if idx is not None else None, _dev(ws, torch.uint8, "ws"), need,
        _stream()))
    return mean, cnt, idx


# -------------------------------------------------------------- two-tower
def tt_params(d, tensors):
    """Build the hrec_tt_params block from a dict of device f32 tensors (the
    caller keeps the tensors alive)."""
    p = TTParams()
    p.d = int(d)
    for name, _ in TTParams._fields_[2:]:
        setattr(p, name, _dev(tensors[name], torch.float32, name).value)
    return p


def tt_item_forward(params, item, man, cat, numeric, out=None):
    n = item.numel()
    if out is None:
        out = torch.empty((n, params.d), dtype=torch.float32, device=item.device)
    elif tuple(out.shape) != (n, params.d):
        raise HrecError(f"tt_item_forward: out must be [{n}, {params.d}], got {tuple(out.shape)}")
    _check("hrec_tt_item_forward", lib().hrec_tt_item_forward(
        ctypes.byref(params), _dev(item, torch.int32, "item"), _dev(man, torch.int32, "manufacturer"),
        _dev(cat, torch.int32, "category"), _dev(numeric, torch.float32, "numeric"), n,
        _dev(out, torch.float32, "item_vec"), _stream()))
    return out


def tt_user_forward(params, user):
    n = user.numel()
    out = torch.empty((n, params.d), dtype=torch.float32, device=user.device)
    _check("hrec_tt_user_forward", lib().hrec_tt_user_forward(
        ctypes.byref(params), _dev(user, torch.int32, "user"), n, _dev(out, torch.float32, "user_vec"),
        _stream()))
    return out


def tt_score(user_vec, item_vec):
    B, d = user_vec.shape
    N = item_vec.shape[0]
    out = torch.empty((B, N), dtype=torch.float32, device=user_vec.device)
    _check("hrec_tt_score", lib().hrec_tt_score(
        _dev(user_vec, torch.float32, "user_vec"), B, _dev(item_vec, torch.float32, "item_vec"), N, d,
        _dev(out, torch.float32, "out"), _stream()))
    return out


# ------------------------------------------------- matrix-core dot + top-k
DOT_DK = (32, 64, 128, 256)


def dot_dk(d):
    """Row width the dot kernels read (d zero-padded up to 32/64/128/256)."""
    for dk in DOT_DK:
        if d <= dk:
            return dk
    raise HrecError(f"dot: vector width {d} > 256 is not supported")


def to_bf16(x):
    """f32 device tensor -> bfloat16 tensor (round to nearest even, on the device)."""
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    _check("hrec_f32_to_bf16", lib().hrec_f32_to_bf16(
        _dev(x, torch.float32, "in"), x.numel(), _vp(out.data_ptr()), _stream()))
    return out


def dot_operand(x, dtype=torch.float32, dk=None):
    """[n, d] f32 vectors -> the kernels' operand: rows of dot_dk(d) (or dk)
    elements, zero-padded, in f32 or bf16 (16-B aligned, contiguous)."""
    n, d = x.shape
    dk = dot_dk(d) if dk is None else int(dk)
    if dk < d:
        raise HrecError(f"dot_operand: dk {dk} < width {d}")
    if d != dk or not x.is_contiguous():
        padded = torch.zeros((n, dk), dtype=x.dtype, device=x.device)
        padded[:, :d] = x
        x = padded
    if dtype == torch.bfloat16:
        return x if x.dtype == torch.bfloat16 else to_bf16(x)
    if x.dtype != torch.float32:
        raise HrecError(f"dot_operand: expected float32, got {x.dtype}")
    return x


def _dot_args(U, V):
    if U.dtype != V.dtype or U.dtype not in (torch.float32, torch.bfloat16):
        raise HrecError("dot: operands must both be float32 or both bfloat16 (see dot_operand)")
    if U.shape[1] != V.shape[1] or U.shape[1] not in DOT_DK:
        raise HrecError(f"dot: operand widths {U.shape[1]} / {V.shape[1]} must match and be one of {DOT_DK}")
    for t, name in ((U, "user_vec"), (V, "item_vec")):
        if not t.is_cuda or not t.is_contiguous():
            raise HrecError(f"dot: {name} must be a contiguous device tensor")
    return U.shape[1], int(U.dtype == torch.bfloat16)


def dot_scores(U, V):
    """out[b, j] = <U[b], V[j]> on the matrix cores (f32 accumulation).
    U, V: operands from dot_operand (same dtype and width)."""
    dk, bf = _dot_args(U, V)
    B, N = U.shape[0], V.shape[0]
    out = torch.empty((B, N), dtype=torch.float32, device=U.device)
    _check("hrec_dot_scores", lib().hrec_dot_scores(
        _vp(U.data_ptr()), B, _vp(V.data_ptr()), N, dk, bf, _dev(out, torch.float32, "out"), N, _stream()))
    return out


DOT_USER_CHUNK = 4096


def dot_topk(U, V, top_k, idx_offset=0, max_rounds=2):
    """Stable top-k of <U[b], V[j]> over all j, never materialising the score
    matrix (hrec_dot_topk). Ties -> smaller j. Returns (idx int64 [B, kk]
    (+ idx_offset), val f32 [B, kk]), kk = min(top_k, N). When a user's
    survivor list overflows, the k-th best of the survivors (a valid, higher
    lower bound) seeds another round; after max_rounds the exact chunked path
    (scores + top-k per chunk + keyed merge) answers."""
    dk, bf = _dot_args(U, V)
    B, N = U.shape[0], V.shape[0]
    kk = min(int(top_k), int(N))
    dev = U.device
    out_i = torch.empty((B, kk), dtype=torch.int64, device=dev)
    out_v = torch.empty((B, kk), dtype=torch.float32, device=dev)
    if B == 0 or kk == 0:
        return out_i, out_v
    for b0 in range(0, B, DOT_USER_CHUNK):
        b1 = min(B, b0 + DOT_USER_CHUNK)
        Ub = U[b0:b1]
        nb = b1 - b0
        need = int(lib().hrec_dot_topk_workspace_bytes(nb, N, kk))
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        oi, ov = out_i[b0:b1], out_v[b0:b1]
        thr = None
        for _ in range(max_rounds):
            _check("hrec_dot_topk", lib().hrec_dot_topk(
                _vp(Ub.data_ptr()), nb, _vp(V.data_ptr()), N, dk, bf, kk,
                None if thr is None else _dev(thr, torch.float32, "thr"), int(idx_offset),
                _dev(oi, torch.int64, "out_idx"), _dev(ov, torch.float32, "out_val"),
                _dev(flag, torch.int32, "overflow"), _dev(ws, torch.uint8, "ws"), need, _stream()))
            if int(flag.item()) == 0:
                break
            thr = ov[:, kk - 1].contiguous()
        else:
            ci, cv = _dot_topk_chunked(Ub, V, kk, idx_offset)
            oi.copy_(ci)
            ov.copy_(cv)
    return out_i, out_v


def dot_filter(U, V, thr, thr_per=0, cap=8192):
    """Survivors of <U[b], V[j]> >= thr[b, j // thr_per] (thr [B] or [B, G]
    f32; thr_per = 0: one bound per user) — hrec_dot_filter. Returns (val f32
    [B, cap], idx int64 [B, cap], count int32 [B]); count > cap = overflow,
    list order unspecified."""
    dk, bf = _dot_args(U, V)
    B, N = U.shape[0], V.shape[0]
    dev = U.device
    thr = thr.to(device=dev, dtype=torch.float32)
    thr = thr.reshape(B, -1).contiguous()
    cv = torch.empty((B, cap), dtype=torch.float32, device=dev)
    ci = torch.empty((B, cap), dtype=torch.int64, device=dev)
    cn = torch.zeros(B, dtype=torch.int32, device=dev)
    _check("hrec_dot_filter", lib().hrec_dot_filter(
        _vp(U.data_ptr()), B, _vp(V.data_ptr()), N, dk, bf, _dev(thr, torch.float32, "thr"), thr.shape[1],
        int(thr_per), int(cap), _vp(cv.data_ptr()), _vp(ci.data_ptr()), _vp(cn.data_ptr()), _stream()))
    return cv, ci, cn


def hybrid_scores(als_users, als_rows, tt_users, als_item, tt_item):
    """Both bf16 score matrices of a hybrid batch and their per-row min/max
    in one launch (hrec_hybrid_scores): als_users [n, ka] f32 ALS factors
    (rows als_rows [B] int64 are used), tt_users [B, kt] f32 two-tower user
    vectors, als_item / tt_item bf16 [N, dk] item operands (dot_operand).
    Returns (als [B, N] f32, tt [B, N] f32, als_mm [2, B], tt_mm [2, B]) —
    dot_scores of the bf16 user operands and rows_minmax of each. A row of
    als_rows outside [0, als_users.shape[0]) gives a NaN ALS score row (as
    als_score does for an unknown user)."""
    dk = _hyb_args(als_item, tt_item)
    B, N = int(als_rows.shape[0]), int(als_item.shape[0])
    if tt_item.shape[0] != N or tt_users.shape[0] != B:
        raise HrecError("hybrid_scores: item counts / batch sizes differ")
    for t, name in ((als_users, "als_users"), (tt_users, "tt_users")):
        if t.dtype != torch.float32 or not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
            raise HrecError(f"hybrid_scores: {name} must be a row-major float32 device matrix")
        if t.shape[1] > dk:
            raise HrecError(f"hybrid_scores: {name} width {t.shape[1]} > operand width {dk}")
    rows = als_rows.to(torch.int64).contiguous()
    dev = als_item.device
    als = torch.empty((B, N), dtype=torch.float32, device=dev)
    tt = torch.empty((B, N), dtype=torch.float32, device=dev)
    a_mm = torch.empty((2, B), dtype=torch.float32, device=dev)
    t_mm = torch.empty((2, B), dtype=torch.float32, device=dev)
    need = int(lib().hrec_hybrid_scores_workspace_bytes(B, N))
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _check("hrec_hybrid_scores", lib().hrec_hybrid_scores(
        _vp(als_users.data_ptr()), als_users.stride(0), _vp(rows.data_ptr()), als_users.shape[0], als_users.shape[1],
        _vp(tt_users.data_ptr()), tt_users.stride(0), tt_users.shape[1], B, _vp(als_item.data_ptr()),
        _vp(tt_item.data_ptr()), N, dk, _vp(als.data_ptr()), _vp(tt.data_ptr()), N, _vp(a_mm.data_ptr()),
        _vp(t_mm.data_ptr()), _vp(ws.data_ptr()), need, _stream()))
    return als, tt, a_mm, t_mm


PRUNE_MAX_K = 8


class HybridPrune:
    """The pruned bf16 hybrid top-k (hrec_hybrid_prune_*) for one batch
    shape: minmax() -> (als_mm, tt_mm) [2, B] (all-reduce them across item
    shards), then topk(als_mm, tt_mm, als_wins, top_k, idx_offset) -> (ids
    [B, kk] int64, fused f64 [B, kk]). Same user / item arguments as
    hybrid_scores; the workspace carries phase 1 into phase 2."""

    def __init__(self, als_users, als_rows, tt_users, als_item, tt_item, top_k):
        self.dk = _hyb_args(als_item, tt_item)
        self.B, self.N = int(als_rows.shape[0]), int(als_item.shape[0])
        if tt_item.shape[0] != self.N or tt_users.shape[0] != self.B:
            raise HrecError("hybrid_prune: item counts / batch sizes differ")
        for t, name in ((als_users, "als_users"), (tt_users, "tt_users")):
            if t.dtype != torch.float32 or not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
                raise HrecError(f"hybrid_prune: {name} must be a row-major float32 device matrix")
            if t.shape[1] > self.dk:
                raise HrecError(f"hybrid_prune: {name} width {t.shape[1]} > operand width {self.dk}")
        if not 1 <= int(top_k) <= PRUNE_MAX_K:
            raise HrecError(f"hybrid_prune: top_k must be in [1, {PRUNE_MAX_K}]")
        self.top_k = int(top_k)
        self.kk = min(self.top_k, self.N)
        self.U, self.rows, self.T = als_users, als_rows.to(torch.int64).contiguous(), tt_users
        self.Va, self.Vt = als_item, tt_item
        dev = als_item.device
        self.need = int(lib().hrec_hybrid_prune_workspace_bytes(self.B, self.N, self.dk, self.top_k))
        self.ws = torch.empty(self.need, dtype=torch.uint8, device=dev)

    def rebind(self, als_rows, tt_users):
        """The same batch shape with other users (the workspace is reused)."""
        if int(als_rows.shape[0]) != self.B or tuple(tt_users.shape) != tuple(self.T.shape) or \
                tt_users.dtype != torch.float32 or tt_users.stride(1) != 1 or not tt_users.is_cuda:
            raise HrecError("hybrid_prune.rebind: batch shape differs from the one the workspace was sized for")
        self.rows = als_rows if als_rows.dtype == torch.int64 and als_rows.is_contiguous() else \
            als_rows.to(torch.int64).contiguous()
        self.T = tt_users
        return self

    def _users(self):
        return (_vp(self.U.data_ptr()), self.U.stride(0), _vp(self.rows.data_ptr()), self.U.shape[0], self.U.shape[1],
                _vp(self.T.data_ptr()), self.T.stride(0), self.T.shape[1], self.B, _vp(self.Va.data_ptr()),
                _vp(self.Vt.data_ptr()), self.N, self.dk)

    def minmax(self):
        dev = self.Va.device
        a_mm = torch.empty((2, self.B), dtype=torch.float32, device=dev)
        t_mm = torch.empty((2, self.B), dtype=torch.float32, device=dev)
        _check("hrec_hybrid_prune_minmax", lib().hrec_hybrid_prune_minmax(
            *self._users(), _vp(a_mm.data_ptr()), _vp(t_mm.data_ptr()), _vp(self.ws.data_ptr()), self.need,
            _stream()))
        return a_mm, t_mm

    def topk(self, als_mm, tt_mm, als_wins, idx_offset=0):
        dev = self.Va.device
        out_i = torch.empty((self.B, self.kk), dtype=torch.int64, device=dev)
        out_v = torch.empty((self.B, self.kk), dtype=torch.float64, device=dev)
        _check("hrec_hybrid_prune_topk", lib().hrec_hybrid_prune_topk(
            *self._users(), _dev(als_mm, torch.float32, "als_mm"), _dev(tt_mm, torch.float32, "tt_mm"),
            int(bool(als_wins)), self.top_k, int(idx_offset), _vp(out_i.data_ptr()), _vp(out_v.data_ptr()),
            _vp(self.ws.data_ptr()), self.need, _stream()))
        return out_i, out_v

    def local(self, als_wins, idx_offset=0):
        """Both phases for ONE item shard (hrec_hybrid_prune_local): the same
        (ids, fused) as minmax() + topk() with one launch fewer; returns
        (ids, fused, als_mm, tt_mm)."""
        dev = self.Va.device
        a_mm = torch.empty((2, self.B), dtype=torch.float32, device=dev)
        t_mm = torch.empty((2, self.B), dtype=torch.float32, device=dev)
        out_i = torch.empty((self.B, self.kk), dtype=torch.int64, device=dev)
        out_v = torch.empty((self.B, self.kk), dtype=torch.float64, device=dev)
        _check("hrec_hybrid_prune_local", lib().hrec_hybrid_prune_local(
            *self._users(), int(bool(als_wins)), self.top_k, int(idx_offset), _vp(a_mm.data_ptr()),
            _vp(t_mm.data_ptr()), _vp(out_i.data_ptr()), _vp(out_v.data_ptr()), _vp(self.ws.data_ptr()), self.need,
            _stream()))
        return out_i, out_v, a_mm, t_mm

    def survivors(self):
        """Survivors of the last topk()'s heavy-model filter per user (int32 [B])."""
        out = torch.empty(self.B, dtype=torch.int32, device=self.Va.device)
        _check("hrec_hybrid_prune_survivors", lib().hrec_hybrid_prune_survivors(
            _vp(self.ws.data_ptr()), self.B, self.N, self.dk, self.top_k, _vp(out.data_ptr()), _stream()))
        return out

    def fallback_taken(self):
        """Whether the last topk() took the exact unfused path (device flag)."""
        out = torch.empty(1, dtype=torch.int32, device=self.Va.device)
        _check("hrec_hybrid_prune_fallback_taken", lib().hrec_hybrid_prune_fallback_taken(
            _vp(self.ws.data_ptr()), self.B, self.N, self.dk, self.top_k, _vp(out.data_ptr()), _stream()))
        return bool(int(out.item()))


EXACT_MAX_K = 8
EXACT_TT_WIDTHS = (32, 64, 128)


def exact_dk(als_width, tt_width):
    """The bf16 operand width of the exact pruned hybrid (64 or 128), or None
    when the shapes are outside it (the materialised path answers)."""
    if tt_width not in EXACT_TT_WIDTHS or not 1 <= als_width <= 128:
        return None
    return 64 if max(als_width, tt_width) <= 64 else 128


class HybridExactItems:
    """One item shard prepared for the exact pruned hybrid
    (hrec_hybrid_exact_prepare): the ALS item factors TRANSPOSED as
    hrec_als_score takes them (Vt [>= k, ld], ld >= n), the two-tower item
    vectors [n, d] (d in 32/64/128, row stride a multiple of 4) and their
    transpose, and the split-bf16 operands + norm bounds of both."""

    def __init__(self, Vt, n_items, k, tt_items):
        self.k, self.d, self.N = int(k), int(tt_items.shape[1]), int(n_items)
        self.dk = exact_dk(self.k, self.d)
        if self.dk is None:
            raise HrecError(f"hybrid_exact: widths (k={self.k}, d={self.d}) outside the exact pruned path")
        for t, name in ((Vt, "Vt"), (tt_items, "tt_items")):
            if t.dtype != torch.float32 or not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
                raise HrecError(f"hybrid_exact: {name} must be a row-major float32 device matrix")
        if Vt.shape[0] < self.k or Vt.stride(0) < self.N or tt_items.shape[0] != self.N:
            raise HrecError("hybrid_exact: Vt must be [>= k, >= n_items] and tt_items [n_items, d]")
        if tt_items.stride(0) % 4 or tt_items.data_ptr() % 16:
            raise HrecError("hybrid_exact: tt_items rows must be 16-B aligned (row stride a multiple of 4)")
        self.Vat, self.Vt = Vt, tt_items
        self.Vtt = transpose(tt_items.contiguous())  # [d, ld]
        self.buf = torch.empty(int(lib().hrec_hybrid_exact_items_bytes(self.N, self.dk)), dtype=torch.uint8,
                               device=tt_items.device)
        _check("hrec_hybrid_exact_prepare", lib().hrec_hybrid_exact_prepare(
            _vp(Vt.data_ptr()), Vt.stride(0), self.k, _vp(tt_items.data_ptr()), tt_items.stride(0), self.d, self.N,
            self.dk, _vp(self.buf.data_ptr()), _stream()))


class HybridExact:
    """The exact pruned hybrid top-k (hrec_hybrid_exact_*) for one batch shape:
    minmax() -> (als_mm, tt_mm) [2, B] (all-reduce them across item shards),
    then topk(als_mm, tt_mm, als_wins, idx_offset) -> (ids [B, kk] int64,
    fused f64 [B, kk]); local() does both for one shard. Bit for bit
    als_score + tt_score + rows_minmax + fuse_rows_topk (batches of >= 8
    users). als_users [n, >= k] f32 (rows als_rows [B] int64 used), tt_users
    [B, d] f32; items: a HybridExactItems."""

    def __init__(self, als_users, als_rows, tt_users, items, top_k):
        if not 1 <= int(top_k) <= EXACT_MAX_K:
            raise HrecError(f"hybrid_exact: top_k must be in [1, {EXACT_MAX_K}]")
        for t, name in ((als_users, "als_users"), (tt_users, "tt_users")):
            if t.dtype != torch.float32 or not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
                raise HrecError(f"hybrid_exact: {name} must be a row-major float32 device matrix")
        if als_users.shape[1] < items.k or tt_users.shape[1] != items.d:
            raise HrecError("hybrid_exact: user widths differ from the prepared items'")
        self.items = items
        self.B, self.N, self.dk = int(als_rows.shape[0]), items.N, items.dk
        if tt_users.shape[0] != self.B:
            raise HrecError("hybrid_exact: batch sizes differ")
        self.top_k = int(top_k)
        self.kk = min(self.top_k, self.N)
        self.U = als_users
        self.need = int(lib().hrec_hybrid_exact_workspace_bytes(self.B, self.N, self.dk))
        self.ws = torch.empty(self.need, dtype=torch.uint8, device=tt_users.device)
        self.rebind(als_rows, tt_users)

    def rebind(self, als_rows, tt_users):
        """The same batch shape with other users (the workspace is reused)."""
        if int(als_rows.shape[0]) != self.B or tuple(tt_users.shape) != (self.B, self.items.d) or \
                tt_users.dtype != torch.float32 or tt_users.stride(1) != 1 or not tt_users.is_cuda:
            raise HrecError("hybrid_exact.rebind: batch shape differs from the one the workspace was sized for")
        self.rows = als_rows if als_rows.dtype == torch.int64 and als_rows.is_contiguous() else \
            als_rows.to(torch.int64).contiguous()
        self.T = tt_users
        it = self.items
        self.arg = HybridBatch(_vp(self.U.data_ptr()), _vp(self.rows.data_ptr()), _vp(self.T.data_ptr()),
                               _vp(it.Vat.data_ptr()), _vp(it.Vt.data_ptr()), _vp(it.Vtt.data_ptr()),
                               _vp(it.buf.data_ptr()), self.U.stride(0), self.U.shape[0], self.T.stride(0),
                               it.Vat.stride(0), it.Vt.stride(0), it.Vtt.stride(0), self.N, it.k, it.d, self.B,
                               self.dk)
        return self

    def _mm(self):
        dev = self.ws.device
        return (torch.empty((2, self.B), dtype=torch.float32, device=dev),
                torch.empty((2, self.B), dtype=torch.float32, device=dev))

    def _out(self):
        dev = self.ws.device
        return (torch.empty((self.B, self.kk), dtype=torch.int64, device=dev),
                torch.empty((self.B, self.kk), dtype=torch.float64, device=dev))

    def minmax(self):
        a_mm, t_mm = self._mm()
        _check("hrec_hybrid_exact_minmax", lib().hrec_hybrid_exact_minmax(
            ctypes.byref(self.arg), _vp(a_mm.data_ptr()), _vp(t_mm.data_ptr()), _vp(self.ws.data_ptr()), self.need,
            _stream()))
        return a_mm, t_mm

    def topk(self, als_mm, tt_mm, als_wins, idx_offset=0):
        out_i, out_v = self._out()
        _check("hrec_hybrid_exact_topk", lib().hrec_hybrid_exact_topk(
            ctypes.byref(self.arg), _dev(als_mm, torch.float32, "als_mm"), _dev(tt_mm, torch.float32, "tt_mm"),
            int(bool(als_wins)), self.top_k, int(idx_offset), _vp(out_i.data_ptr()), _vp(out_v.data_ptr()),
            _vp(self.ws.data_ptr()), self.need, _stream()))
        return out_i, out_v

    def local(self, als_wins, idx_offset=0):
        """Both phases for ONE item shard: (ids, fused, als_mm, tt_mm)."""
        a_mm, t_mm = self._mm()
        out_i, out_v = self._out()
        _check("hrec_hybrid_exact_local", lib().hrec_hybrid_exact_local(
            ctypes.byref(self.arg), int(bool(als_wins)), self.top_k, int(idx_offset), _vp(a_mm.data_ptr()),
            _vp(t_mm.data_ptr()), _vp(out_i.data_ptr()), _vp(out_v.data_ptr()), _vp(self.ws.data_ptr()), self.need,
            _stream()))
        return out_i, out_v, a_mm, t_mm

    def counts(self):
        """(groups rescored per user for the extremes [B], for the top-k [B],
        whether some user rescored every group) of the last call."""
        out = torch.empty(2 * self.B + 1, dtype=torch.int32, device=self.ws.device)
        _check("hrec_hybrid_exact_counts", lib().hrec_hybrid_exact_counts(
            _vp(self.ws.data_ptr()), self.B, self.N, self.dk, _vp(out.data_ptr()), _stream()))
        return out[: self.B], out[self.B: 2 * self.B], bool(int(out[2 * self.B].item()))


def _hyb_args(*ops):
    dk = ops[0].shape[1]
    for t in ops:
        if t.dtype != torch.bfloat16 or t.shape[1] != dk or not t.is_cuda or not t.is_contiguous():
            raise HrecError("hybrid: operands must be contiguous bfloat16 device tensors of one width")
    if dk not in (64, 128, 256):
        raise HrecError(f"hybrid: width {dk} must be 64, 128 or 256")
    return dk


def _dot_topk_chunked(U, V, kk, idx_offset, chunk=1 << 20):
    """Exact fallback: dot_scores per item chunk, per-chunk stable top-k with
    global ids, keyed merge (ties -> smaller id)."""
    cand_i, cand_v = [], []
    for j0 in range(0, V.shape[0], chunk):
        s = dot_scores(U, V[j0:j0 + chunk])
        i, v = topk(s, kk)
        cand_i.append(i + (j0 + idx_offset))
        cand_v.append(v.double())
    ci = torch.cat(cand_i, 1).contiguous()
    cv = torch.cat(cand_v, 1).contiguous()
    i, v = topk_keyed(cv, ci, kk)
    return i, v.float()


def tt_pair_score(user_vec, item_vec):
    n, d = user_vec.shape
    out = torch.empty(n, dtype=torch.float32, device=user_vec.device)
    _check("hrec_tt_pair_score", lib().hrec_tt_pair_score(
        _dev(user_vec, torch.float32, "user_vec"), _dev(item_vec, torch.float32, "item_vec"), n, d,
        _dev(out, torch.float32, "out"), _stream()))
    return out


TT_INPUTS_IDS, TT_INPUTS_INF, TT_INPUTS_DUP = 1, 2, 4


def tt_item_inputs(item, man, cat, price, rating, tables, scale, min_, ws=None):
    """hrec_tt_item_inputs: device int64 id columns + f64 numeric columns ->
    (item, man, cat int32 [n], numeric f32 [n, 2], flags int32 [1] device).
    tables = (n_item, n_man, n_cat); scale / min_: the scaler's 2 doubles.
    flags != 0: an id outside its table (or >= 2^24), an infinite numeric
    value or a repeated item id — the outputs are then not the model's
    inputs. ws: a reusable uint8 workspace of
    hrec_tt_item_inputs_workspace_bytes(n_item) bytes."""
    n = item.numel()
    dev = item.device
    need = int(lib().hrec_tt_item_inputs_workspace_bytes(int(tables[0])))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3)]
    num = torch.empty((n, 2), dtype=torch.float32, device=dev)
    flags = torch.empty(1, dtype=torch.int32, device=dev)
    sc = (ctypes.c_double * 2)(float(scale[0]), float(scale[1]))
    mn = (ctypes.c_double * 2)(float(min_[0]), float(min_[1]))
    _check("hrec_tt_item_inputs", lib().hrec_tt_item_inputs(
        _dev(item, torch.int64, "item"), _dev(man, torch.int64, "man"), _dev(cat, torch.int64, "cat"),
        _dev(price, torch.float64, "price"), _dev(rating, torch.float64, "rating"), n, int(tables[0]),
        int(tables[1]), int(tables[2]), ctypes.cast(sc, _vp), ctypes.cast(mn, _vp), _vp(outs[0].data_ptr()),
        _vp(outs[1].data_ptr()), _vp(outs[2].data_ptr()), _vp(num.data_ptr()), _vp(flags.data_ptr()),
        _vp(ws.data_ptr()), ws.numel(), _stream()))
    return outs[0], outs[1], outs[2], num, flags, ws


def tt_grad_len(d):
    return int(lib().hrec_tt_grad_len(int(d)))


def tt_forward_backward(params, user, item, man, cat, numeric, y, ws=None):
    """Returns (grad_dense [grad_len], g_user, g_item, g_man, g_cat)."""
    B = user.numel()
    d = params.d
    dev = user.device
    need = int(lib().hrec_tt_train_workspace_bytes(d, B))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
    gd = torch.empty(tt_grad_len(d), dtype=torch.float32, device=dev)
    gu = torch.empty((B, d), dtype=torch.float32, device=dev)
    gi = torch.empty((B, d), dtype=torch.float32, device=dev)
    gm = torch.empty((B, 8), dtype=torch.float32, device=dev)
    gc = torch.empty((B, 8), dtype=torch.float32, device=dev)
    _check("hrec_tt_forward_backward", lib().hrec_tt_forward_backward(
        ctypes.byref(params), _dev(user, torch.int32, "user"), _dev(item, torch.int32, "item"),
        _dev(man, torch.int32, "manufacturer"), _dev(cat, torch.int32, "category"),
        _dev(numeric, torch.float32, "numeric"), _dev(y, torch.float32, "y"), B,
        _dev(gd, torch.float32, "grad_dense"), _dev(gu, torch.float32, "g_user"),
        _dev(gi, torch.float32, "g_item"), _dev(gm, torch.float32, "g_man"), _dev(gc, torch.float32, "g_cat"),
        _dev(ws, torch.uint8, "workspace"), ws.numel(), _stream()))
    return gd, gu, gi, gm, gc


def adam_dense(var, m, v, grad, alpha, beta1, beta2, eps):
    _check("hrec_adam_dense", lib().hrec_adam_dense(
        _dev(var, torch.float32, "var"), _dev(m, torch.float32, "m"), _dev(v, torch.float32, "v"),
        _dev(grad, torch.float32, "grad"), var.numel(), float(alpha), float(beta1), float(beta2), float(eps),
        _stream()))


def adam_sparse(var, m, v, indices, grad_rows, mark, gsum, lr, beta1, omb1, beta2, omb2, eps):
    n_rows, dim = var.shape
    _check("hrec_adam_sparse", lib().hrec_adam_sparse(
        _dev(var, torch.float32, "var"), _dev(m, torch.float32, "m"), _dev(v, torch.float32, "v"), n_rows, dim,
        _dev(indices, torch.int32, "indices"), _dev(grad_rows, torch.float32, "grad_rows"), indices.numel(),
        _dev(mark, torch.int32, "mark"), _dev(gsum, torch.float32, "gsum"), float(lr), float(beta1),
        float(omb1), float(beta2), float(omb2), float(eps), _stream()))


def adam_sparse_tables(tables, lr, beta1, omb1, beta2, omb2, eps):
    """hrec_adam_sparse over several tables in 3 launches. tables: list of
    (var, m, v, indices, grad_rows, mark, gsum) tuples, as adam_sparse takes."""
    if len(tables) > MAX_SPARSE_TABLES:
        raise HrecError(f"adam_sparse_tables: at most {MAX_SPARSE_TABLES} tables")
    arr = (SparseTable * max(1, len(tables)))()
    for j, (var, m, v, indices, grad_rows, mark, gsum) in enumerate(tables):
        n_rows, dim = var.shape
        arr[j] = SparseTable(_dev(var, torch.float32, "var"), _dev(m, torch.float32, "m"),
                             _dev(v, torch.float32, "v"), n_rows, dim, indices.numel(),
                             _dev(indices, torch.int32, "indices"), _dev(grad_rows, torch.float32, "grad_rows"),
                             _dev(mark, torch.int32, "mark"), _dev(gsum, torch.float32, "gsum"))
    _check("hrec_adam_sparse_tables", lib().hrec_adam_sparse_tables(
        arr, len(tables), float(lr), float(beta1), float(omb1), float(beta2), float(omb2), float(eps), _stream()))


SPARSE_MARK, SPARSE_SWEEP_UNTOUCHED, SPARSE_TOUCHED, SPARSE_UNMARK = 0, 1, 2, 3


def sparse_tables_arg(tables):
    """ctypes array of hrec_sparse_table for the phased sparse Adam: tables is
    a list of (var, m, v, indices, grad_rows, mark) (no gsum: phase 2 sums
    the gradients in registers). Build once per step, pass to every phase."""
    if len(tables) > MAX_SPARSE_TABLES:
        raise HrecError(f"adam_sparse_tables_phase: at most {MAX_SPARSE_TABLES} tables")
    arr = (SparseTable * max(1, len(tables)))()
    for j, (var, m, v, indices, grad_rows, mark) in enumerate(tables):
        n_rows, dim = var.shape
        arr[j] = SparseTable(_dev(var, torch.float32, "var"), _dev(m, torch.float32, "m"),
                             _dev(v, torch.float32, "v"), n_rows, dim, indices.numel(),
                             _dev(indices, torch.int32, "indices"), _dev(grad_rows, torch.float32, "grad_rows"),
                             _dev(mark, torch.int32, "mark"), None)
    return arr, len(tables)


def adam_sparse_tables_phase(arg, phase, lr=0.0, beta1=0.0, omb1=0.0, beta2=0.0, omb2=0.0, eps=0.0):
    """One phase of hrec_adam_sparse_tables_phase on the current stream
    (arg from sparse_tables_arg)."""
    arr, n = arg
    _check("hrec_adam_sparse_tables_phase", lib().hrec_adam_sparse_tables_phase(
        arr, n, int(phase), float(lr), float(beta1), float(omb1), float(beta2), float(omb2), float(eps),
        _stream()))


# --------------------------------------------------------- batched fusion
def rows_minmax(x):
    n_rows, n = x.shape
    out = torch.empty((2, n_rows), dtype=torch.float32, device=x.device)  # [mins; maxes]
    _check("hrec_rows_minmax_f32", lib().hrec_rows_minmax_f32(
        _dev(x, torch.float32, "x"), n_rows, n, x.stride(0), _dev(out, torch.float32, "out"), _stream()))
    return out


def fuse_rows_topk(als, tt, als_mm, tt_mm, als_wins, top_k, idx_offset=0):
    n_rows, n = als.shape
    kk = min(int(top_k), n)
    dev = als.device
    out_i = torch.empty((n_rows, kk), dtype=torch.int64, device=dev)
    out_v = torch.empty((n_rows, kk), dtype=torch.float64, device=dev)
    need = int(lib().hrec_fuse_rows_workspace_bytes(n_rows, n, kk))
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _check("hrec_fuse_rows_topk", lib().hrec_fuse_rows_topk(
        _dev(als, torch.float32, "als"), _dev(tt, torch.float32, "tt"), n_rows, n, als.stride(0),
        _dev(als_mm, torch.float32, "als_minmax"), _dev(tt_mm, torch.float32, "tt_minmax"), int(bool(als_wins)),
        kk, int(idx_offset), _dev(out_i, torch.int64, "out_idx"), _dev(out_v, torch.float64, "out_val"),
        _dev(ws, torch.uint8, "ws"), need, _stream()))
    return out_i, out_v


def topk_keyed(vals, keys, top_k):
    n_rows, n = vals.shape
    kk = min(int(top_k), n)
    dev = vals.device
    out_i = torch.empty((n_rows, kk), dtype=torch.int64, device=dev)
    out_v = torch.empty((n_rows, kk), dtype=torch.float64, device=dev)
    need = int(lib().hrec_topk_workspace_bytes(n_rows, n, kk, 1))
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _check("hrec_topk_f64_keyed", lib().hrec_topk_f64_keyed(
        _dev(vals, torch.float64, "vals"), _dev(keys, torch.int64, "keys"), n_rows, n, kk,
        _dev(out_i, torch.int64, "out_idx"), _dev(out_v, torch.float64, "out_val"), _dev(ws, torch.uint8, "ws"),
        need, _stream()))
    return out_i, out_v


# ------------------------------------------------------- multi-GPU (C-ABI)
_COMM_DTYPES = {torch.float32: 0, torch.float64: 1, torch.int32: 2, torch.int64: 3, torch.uint8: 4}


class Comm:
    """The C-ABI's RCCL communicator (hrec_comm_*), for hosts that drive the
    exchange steps through libhrec instead of torch.distributed: rank 0's
    unique_id() goes to every rank by the host's own channel, then every
    rank constructs Comm(rank, world, uid)."""

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * 128)()
        _check("hrec_comm_get_unique_id", lib().hrec_comm_get_unique_id(ctypes.cast(buf, _vp)))
        return bytes(buf)

    def __init__(self, rank, world, uid):
        if len(uid) != 128:
            raise HrecError("Comm: the unique id has 128 bytes")
        self._id = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self.h = _vp()
        self.rank, self.world = int(rank), int(world)
        _check("hrec_comm_init", lib().hrec_comm_init(self.rank, self.world, ctypes.cast(self._id, _vp),
                                                      ctypes.byref(self.h)))

    def allgather(self, send, recv=None):
        """recv [world * n] = every rank's send [n] (rank-major)."""
        if send.dtype not in _COMM_DTYPES or not send.is_cuda or not send.is_contiguous():
            raise HrecError("Comm.allgather: a contiguous device tensor of f32/f64/i32/i64/u8")
        if recv is None:
            recv = torch.empty((self.world,) + tuple(send.shape), dtype=send.dtype, device=send.device)
        elif recv.numel() != self.world * send.numel() or recv.device != send.device:
            # hrec_allgather writes world x count elements: a smaller buffer is an out-of-bounds write
            raise HrecError(f"Comm.allgather: recv holds {recv.numel()} elements on {recv.device}, "
                            f"need {self.world} x {send.numel()} on {send.device}")
        _check("hrec_allgather", lib().hrec_allgather(self.h, _vp(send.data_ptr()), _dev(recv, send.dtype, "recv"),
                                                      send.numel(), _COMM_DTYPES[send.dtype], _stream()))
        return recv

    def allreduce_minmax(self, mm):
        """mm [n_rows, 2, B] f32 (each model's [min; max]) -> global extremes, in place."""
        if mm.dim() != 3 or mm.shape[1] != 2:
            raise HrecError("Comm.allreduce_minmax: mm must be [n_rows, 2, B]")
        if not mm.is_cuda or mm.dtype != torch.float32:
            raise HrecError("Comm.allreduce_minmax: mm must be a float32 device tensor")
        _check("hrec_allreduce_minmax", lib().hrec_allreduce_minmax(
            self.h, _dev(mm, torch.float32, "mm"), mm.shape[0], mm.shape[2], _stream()))
        return mm

    def close(self):
        if self.h:
            _check("hrec_comm_destroy", lib().hrec_comm_destroy(self.h))
            self.h = _vp()
