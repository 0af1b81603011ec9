"""CPU-side checks of the drop-in boundary: the C-ABI library loads without a
GPU and exports every entry point include/jg.h declares (no compute calls)."""
import os
import re

from cap_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "jg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(jg_[a-z_]+)\s*\(", src)))


def test_header_declares_the_documented_abi():
    syms = declared_symbols()
    for s in ("jg_create", "jg_destroy", "jg_keys_load", "jg_verify_batch", "jg_last_error", "jg_host_alloc",
              "jg_host_free"):
        assert s in syms
    assert sorted(_lib.EXPORTS) == syms


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert b"gfx950" in L.jg_version()


def test_struct_layouts_match_header():
    import ctypes
    assert ctypes.sizeof(_lib.JgTok) == 24
    assert _lib.JgTok.key_idx.offset == 20 and _lib.JgTok.alg.offset == 22
    assert _lib.JgKey.e.offset == 24 and _lib.JgKey.coord_len.offset == 48
    src = open(os.path.join(ROOT, "include", "jg.h")).read()
    assert "uint64_t off;\n  uint32_t len;\n  uint8_t fam;" in src        # jg_hjob: 16 bytes


def test_no_device_fails_loudly():
    """Without a HIP device the product refuses to run (no CPU fallback)."""
    import pytest
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(_lib.JgError):
        _lib.Context()
