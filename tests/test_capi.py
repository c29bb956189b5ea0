"""CPU: librs_hip.so loads, exports every symbol include/*.h declares,
matches the ctypes signature table, and rejects bad arguments before any
device work (these calls launch nothing)."""
import ctypes as C
import os
import re

import pytest

from recommender_system_amd import _lib

INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HDRS = sorted(os.path.join(INC, f) for f in os.listdir(INC) if f.endswith(".h"))


def _headers_text():
    return re.sub(r"/\*.*?\*/", "", "".join(open(h).read() for h in HDRS), flags=re.S)


def declared():
    return sorted(set(re.findall(r"\b(rs_[a-z0-9_]+)\s*\(", _headers_text())))


def test_header_symbols_exported_and_bound():
    lib = _lib.lib()
    names = declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/*.h but not exported"
    assert set(names) == set(_lib.SIGNATURES), "ctypes table out of sync with include/*.h"


def test_version_and_sizes():
    lib = _lib.lib()
    assert b"gfx950" in lib.rs_version()
    n = lib.rs_fm_prepared_size(13, 26, 16, 10)
    assert n == 4 * (64 + 4) + 26 * (64 * 4 + 16)  # dense records + field records
    assert lib.rs_fm_prepared_size(-1, 26, 16, 10) == -1
    assert lib.rs_cross_prepared_size(429, 3) > 108 * 64
    assert lib.rs_shard_workspace_size(4096 * 26, 8) > 0
    assert lib.rs_shard_workspace_size(10, 65) == -1


def test_argument_validation_without_device():
    lib = _lib.lib()
    st = lib.rs_embed_fm_fwd(None, 0, 26, None, 13, 13, None, None, None, 26, 16, None, None, 10, None, None, 4096,
                             None, None)
    assert st == -1 and b"null" in lib.rs_last_error_string()
    assert lib.rs_dense_fwd(None, 4, None, None, None, 0, None, 4, 4, 4, 4, None) == -1
    assert lib.rs_din_attention_fwd(*([C.c_void_p(1)] * 4), 100, 12, *([C.c_void_p(1)] * 3), 80,
                                    *([C.c_void_p(1)] * 3), 40, C.c_void_p(1), C.c_void_p(1), C.c_void_p(1), 8,
                                    None) == -1
    assert b"k must be" in lib.rs_last_error_string()
    assert lib.rs_cross_fwd(C.c_void_p(1), 10, 10, 40, C.c_void_p(1), C.c_void_p(1), 10, 4, None) == -1
    with pytest.raises(_lib.RSError):
        _lib.call("rs_sigmoid_combine", None, None, 1.0, 1.0, None, 4, None)


def test_product_path_has_no_cpu_fallback():
    import torch
    from recommender_system_amd import FMLayer
    layer = FMLayer(4, device="cpu", input_dim=8)
    with pytest.raises(_lib.RSError, match="device"):
        layer(torch.zeros(2, 8))


def test_signature_arity_matches_header():
    txt = _headers_text()
    for m in re.finditer(r"\b(rs_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", txt):
        name, params = m.group(1), m.group(2).strip()
        n = 0 if params in ("", "void") else len(params.split(","))
        assert len(_lib.SIGNATURES[name][1]) == n, f"{name}: header has {n} params"


def test_runtime_options():
    """rs_set_option / rs_get_option: known options round-trip, unknown ones
    and out-of-range values are refused without changing anything."""
    lib = _lib.lib()
    opt = _lib.OPT_EMBED_FM_KERNEL
    cur = lib.rs_get_option(opt)
    assert cur >= 0
    for v in range(4):
        assert lib.rs_set_option(opt, v) >= 0
        assert lib.rs_get_option(opt) == v
    assert lib.rs_set_option(opt, cur) == 3
    assert lib.rs_set_option(opt, 7) == -1 and lib.rs_get_option(opt) == cur
    assert lib.rs_get_option(99) == -1
    assert lib.rs_set_option(-1, 0) == -1 and b"unknown option" in lib.rs_last_error_string()
    with pytest.raises(_lib.RSError):
        _lib.set_option(99, 1)


def test_runtime_options_are_thread_local():
    """ADVICE/VERDICT r4: rs_set_option is per host thread — a setting made on
    one thread neither leaks into another thread's launches nor is changed by
    them, and every thread starts from the defaults (no process-wide mutable
    state behind the C-ABI)."""
    import threading
    lib = _lib.lib()
    opt = _lib.OPT_EMBED_FM_KERNEL
    default = lib.rs_get_option(opt)
    prev = lib.rs_set_option(opt, 2)
    seen = {}

    def other():
        seen["start"] = lib.rs_get_option(opt)
        lib.rs_set_option(opt, 3)
        seen["own"] = lib.rs_get_option(opt)

    try:
        th = threading.Thread(target=other)
        th.start()
        th.join()
        assert seen == {"start": default, "own": 3}
        assert lib.rs_get_option(opt) == 2
    finally:
        lib.rs_set_option(opt, prev)
