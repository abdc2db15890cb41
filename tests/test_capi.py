"""CPU: the C-ABI library builds for gfx950, loads, and exports every entry
point include/hrec.h declares (no compute call without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    with open(os.path.join(ROOT, "include", "hrec.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hrec_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    import __graft_entry__ as g

    lib_path = g.build_lib()
    import torch  # noqa: F401  (binds libamdhip64 first, as the product does)

    lib = ctypes.CDLL(lib_path)
    declared = _declared()
    assert len(declared) >= 20
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    lib.hrec_abi_version.restype = ctypes.c_int
    assert lib.hrec_abi_version() == 7


def test_python_binding_covers_the_header():
    from src import _hrec

    assert set(_declared()) == set(_hrec.exported_symbols())


def test_invalid_arguments_fail_loudly_without_gpu():
    import __graft_entry__ as g

    lib = ctypes.CDLL(g.build_lib())
    lib.hrec_als_half_sweep.restype = ctypes.c_int
    lib.hrec_last_error.restype = ctypes.c_char_p
    rc = lib.hrec_als_half_sweep(None, None, None, ctypes.c_int64(1), None, ctypes.c_int64(1), 8, 48,
                                 ctypes.c_double(0.1), 0, None, None)
    assert rc == -1
    assert b"kp must be 16, 32, 64, 96, 128, 192 or 256" in lib.hrec_last_error()
    # grouped sparse Adam: the table count is checked before any device work
    f = lib.hrec_adam_sparse_tables
    f.restype = ctypes.c_int
    args = [ctypes.c_float(0.001), ctypes.c_float(0.9), ctypes.c_float(0.1), ctypes.c_float(0.999),
            ctypes.c_float(0.001), ctypes.c_float(1e-7), None]
    assert f(None, 9, *args) == -1
    assert b"tables" in lib.hrec_last_error()
    assert f(None, 0, *args) == 0  # nothing to update
    # the RCCL exchange steps: argument checks before RCCL is touched
    lib.hrec_allgather.restype = ctypes.c_int
    assert lib.hrec_allgather(None, None, None, ctypes.c_size_t(4), 0, None) == -1
    assert b"null communicator" in lib.hrec_last_error()
    lib.hrec_comm_init.restype = ctypes.c_int
    idb = (ctypes.c_uint8 * 128)()
    out = ctypes.c_void_p()
    assert lib.hrec_comm_init(2, 2, idb, ctypes.byref(out)) == -1
    assert b"rank 2 of world 2" in lib.hrec_last_error()
    lib.hrec_allreduce_minmax.restype = ctypes.c_int
    assert lib.hrec_allreduce_minmax(ctypes.c_void_p(8), None, 0, ctypes.c_int64(3), None) == -1
    # phased sparse Adam: phase range and table count before any device work
    fp = lib.hrec_adam_sparse_tables_phase
    fp.restype = ctypes.c_int
    assert fp(None, 1, 4, *args) == -1
    assert b"phase 4 not in 0..3" in lib.hrec_last_error()
    assert fp(None, 9, 0, *args) == -1
    assert b"tables" in lib.hrec_last_error()
    assert fp(None, 0, 1, *args) == 0
    # f64-source half-sweep: kp 64 only
    h = lib.hrec_als_half_sweep_src64
    h.restype = ctypes.c_int
    assert h(None, None, None, ctypes.c_int64(1), None, ctypes.c_int64(1), 8, 32, ctypes.c_double(0.1), None,
             None) == -1
    assert b"kp must be 64" in lib.hrec_last_error()
    # bf16 hybrid scores: operand width and workspace are checked first
    hs = lib.hrec_hybrid_scores
    hs.restype = ctypes.c_int
    hs.argtypes = ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                    ctypes.c_int64,
                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
                   + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_void_p])
    assert hs(None, 96, None, 0, 96, None, 96, 96, 4, None, None, 10, 96, None, None, 10, None, None, None, 0, None) == -1
    assert b"dk must be 64, 128 or 256" in lib.hrec_last_error()
    assert hs(None, 64, None, 0, 64, None, 64, 64, 4, None, None, 10, 64, None, None, 10, None, None, None, 0, None) == -1
    assert b"null min/max output or workspace" in lib.hrec_last_error()
    assert hs(None, 64, None, -1, 64, None, 64, 64, 4, None, None, 10, 64, None, None, 10, None, None, None, 0,
              None) == -1
    assert b"negative n_als_rows" in lib.hrec_last_error()
    assert hs(None, 64, None, 0, 64, None, 64, 64, 0, None, None, 10, 64, None, None, 10, None, None, None, 0,
              None) == 0  # no users: nothing to do
    # exact hybrid without score matrices: the batch description is checked first
    from src import _hrec

    ex = lib.hrec_hybrid_exact_minmax
    ex.restype = ctypes.c_int
    ex.argtypes = [ctypes.POINTER(_hrec.HybridBatch)] + [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_void_p]
    assert ex(None, None, None, None, 0, None) == -1
    assert b"null batch" in lib.hrec_last_error()
    bt = _hrec.HybridBatch(None, None, None, None, None, None, None, 64, 10, 64, 128, 64, 128, 100, 64, 64, 4, 96)
    assert ex(ctypes.byref(bt), None, None, None, 0, None) == -1
    assert b"dk must be 64 or 128" in lib.hrec_last_error()
    bt.dk, bt.tt_width = 64, 48
    assert ex(ctypes.byref(bt), None, None, None, 0, None) == -1
    assert b"tt_width must be 32, 64 or 128" in lib.hrec_last_error()
    bt.tt_width, bt.tt_items_ld = 64, 30
    assert ex(ctypes.byref(bt), None, None, None, 0, None) == -1
    assert b"bad item strides" in lib.hrec_last_error()
    bt.tt_items_ld = 64
    assert ex(ctypes.byref(bt), None, None, None, 0, None) == -1
    assert b"null pointer" in lib.hrec_last_error()
    tk = lib.hrec_hybrid_exact_topk
    tk.restype = ctypes.c_int
    tk.argtypes = [ctypes.POINTER(_hrec.HybridBatch), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                   ctypes.c_void_p]
    bt.n_users = 0
    assert tk(ctypes.byref(bt), None, None, 0, 9, 0, None, None, None, 0, None) == -1
    assert b"top_k must be in [1, 8]" in lib.hrec_last_error()
    assert tk(ctypes.byref(bt), None, None, 0, 5, 0, None, None, None, 0, None) == 0  # no users


def test_product_has_no_oracle_imports():
    pkg = os.path.join(ROOT, "hybrid-als-twotower-recommender_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                with open(os.path.join(dirpath, f)) as fh:
                    src = fh.read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f


def test_facade_reexports_reference_classes():
    """src/__init__.py:39-42 of the reference: `from src import ...` works."""
    import src
    from src import ALSModel, HybridRecommendationSystem, RecommenderEvaluator, TwoTowerModel

    assert src.__all__ == ["HybridRecommendationSystem", "ALSModel", "TwoTowerModel", "RecommenderEvaluator"]
    assert ALSModel.__module__ == "src.als_model"
    assert TwoTowerModel.__module__ == "src.two_tower_model"
    assert HybridRecommendationSystem.__module__ == "src.hybrid_system"
    assert RecommenderEvaluator.__module__ == "src.evaluation"


def test_topk_workspace_query_terminates_for_large_k():
    """the workspace query looped forever for top_k > 2048; any
    top_k is now accepted (above 1024 by the device sort path)."""
    import __graft_entry__ as g

    lib = ctypes.CDLL(g.build_lib())
    for fn in ("hrec_topk_workspace_bytes",):
        f = getattr(lib, fn)
        f.restype = ctypes.c_size_t
        f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
        for n, k in ((5000, 3000), (100000, 3000), (100000, 5000), (100000, 1500), (100000, 1024), (10, 3000)):
            assert f(1, n, k, 1) > 0
            assert f(4, n, k, 0) > 0
    f = lib.hrec_fuse_workspace_bytes
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.c_int64, ctypes.c_int]
    assert f(100000, 5000) > 100000 * 8
    f = lib.hrec_fuse_rows_workspace_bytes
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    assert f(2, 100000, 3000) > 0


def test_comm_rccl_enum_values_match_header():
    """csrc/comm.hip restates the few rccl.h enum values it passes (dtype and
    ncclMin) as literals: each must equal the header's value."""
    import re
    hdr = "/opt/rocm/include/rccl/rccl.h"
    if not os.path.exists(hdr):
        pytest.skip("rccl.h not present")
    text = open(hdr).read()
    src = open(os.path.join(ROOT, "hybrid-als-twotower-recommender_amd", "csrc", "comm.hip")).read()
    pairs = re.findall(r"(\d+) /\* (nccl\w+) \*/", src)
    assert {n for _, n in pairs} >= {"ncclFloat32", "ncclFloat64", "ncclInt32", "ncclInt64", "ncclUint8", "ncclMin"}
    for val, name in pairs:
        m = re.search(r"\b%s\s*=\s*(\d+)" % name, text)
        assert m, name
        assert int(val) == int(m.group(1)), (name, val, m.group(1))
