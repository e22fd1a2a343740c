"""CPU: libposekern.so loads and exports every entry point include/posekern.h declares,
and the ctypes table mirrors the header."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "posekern.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.findall(r"\b(?:int|int64_t)\s+(pk_\w+)\s*\(([^;]*)\)\s*;", src)


def test_header_declares_entry_points():
    names = [n for n, _ in header_functions()]
    assert "pk_fps" in names and "pk_ball_query_mask" in names
    assert len(names) == len(set(names))


def test_library_exports_every_symbol():
    from dpfm_amd import _lib
    lib = _lib.lib()
    for name, args in header_functions():
        assert hasattr(lib, name), name
        nargs = len([a for a in args.split(",") if a.strip()])
        assert name in _lib.SIGNATURES, f"{name} missing from the ctypes table"
        assert len(_lib.SIGNATURES[name]) == nargs, f"{name}: header has {nargs} args"
    assert set(_lib.SIGNATURES) == {n for n, _ in header_functions()}


def test_no_cpu_fallback():
    import torch
    from dpfm_amd import ops, _lib
    x = torch.zeros(10, 3)
    off = torch.tensor([0, 10])
    with pytest.raises(_lib.PoseKernError):
        ops.fps_packed(x, off, 10, torch.zeros(1, dtype=torch.int32), torch.ones(1, dtype=torch.int32), 1)
