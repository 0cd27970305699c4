"""The C-ABI library loads and exports every entry point include/tbg.h declares (no GPU needed)."""
import ctypes
import os
import re

from tigerbeetle_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "tbg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tbg_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_loader_list():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert b"gfx950" in L.tbg_version()


def test_library_is_gfx950_code_object():
    # the HIP fat binary carries a gfx950 code object
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_input_valid_without_device():
    # input_valid needs no device (state_machine.zig:543-572; test at :3573-3665)
    L = _lib.lib()
    for op, size, mx, mn in ((129, 128, 8190, 0), (130, 128, 8190, 0), (131, 16, 8190, 0), (132, 16, 8190, 0)):
        assert L.tbg_input_valid(None, op, 0) == (mn == 0)
        assert L.tbg_input_valid(None, op, size)
        assert L.tbg_input_valid(None, op, mx * size)
        assert not L.tbg_input_valid(None, op, (mx + 1) * size)
        assert not L.tbg_input_valid(None, op, 3 * (size // 2))
    assert L.tbg_input_valid(None, 128, 0) and not L.tbg_input_valid(None, 128, 128)
    assert L.tbg_input_valid(None, 133, 64) and not L.tbg_input_valid(None, 133, 0)
