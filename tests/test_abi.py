"""CPU checks of the C ABI: the product library loads (no GPU needed to load) and
exports every entry point include/mtgpu.h declares; the emulation build exports
the same set under emu_."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    h = open(os.path.join(ROOT, "include", "mtgpu.h")).read()
    return sorted(set(re.findall(r"\b(mt_[a-z0-9_]+)\s*\(", h)))


def test_header_declares_entry_points():
    d = declared()
    for name in ("mt_create", "mt_apply_batch", "mt_snapshot_v1", "mt_get_text", "mt_generate", "mt_get_length"):
        assert name in d


def test_product_library_exports_every_symbol():
    import __graft_entry__
    lib = ctypes.CDLL(__graft_entry__.build_engine())  # rebuilds unless it carries this tree's source hash
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_emulation_library_exports_same_symbols():
    from emu_lib import build_emu
    lib = ctypes.CDLL(build_emu())
    missing = [n for n in declared() if not hasattr(lib, "emu_" + n[3:])]
    assert not missing, missing


def test_product_library_is_built_from_this_tree():
    """The library carries the sha256 of the sources it was compiled from (mt_source_hash):
    a stale libmtgpu.so (older than csrc/ or include/) fails here, on CPU, before any GPU run."""
    import __graft_entry__
    lib = ctypes.CDLL(__graft_entry__.build_engine())
    lib.mt_source_hash.restype = ctypes.c_char_p
    assert lib.mt_source_hash().decode() == __graft_entry__.source_hash()
