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


def test_product_library_has_no_development_hooks():
    """The product libposekern.so exports no pkdev_* hook and reads no environment switch
    (those live in libposekern_dev.so, built from the same sources with -DPK_DEVBUILD); the dev
    library exports the hooks the tests / tools use."""
    import subprocess
    from dpfm_amd import _lib
    nm = lambda p: subprocess.run(["nm", "-D", p], capture_output=True, text=True, check=True).stdout  # noqa: E731
    prod = nm(_lib.LIB_PATH)
    assert "pkdev_" not in prod
    assert not re.search(r"\bU getenv\b", prod)
    dev = nm(_lib.DEV_LIB_PATH)
    for hook in ("pkdev_seq_sum", "pkdev_rigidity_variant", "pkdev_probe_linear", "pkdev_fps_cfg"):
        assert hook in dev, hook


def test_build_id_matches_tree():
    """pk_build_id of the loaded product and dev libraries equals the sha256 recomputed from this
    tree's sources (csrc, include/posekern.h, Makefile): the binaries are built from them."""
    from dpfm_amd import _lib
    want = _lib.tree_build_id()
    assert _lib.build_id() == want, "libposekern.so was not built from this tree (run make)"
    assert _lib.build_id(_lib.dev_lib()) == want, "libposekern_dev.so was not built from this tree (run make)"


@pytest.mark.gpu
def test_build_id_matches_tree_on_device():
    """The same identity check inside the GPU suite (the box runs the .so pushed from the build
    container), after one device call through the library, so a green -m gpu run proves the tested
    binary is built from the snapshot's sources."""
    import torch
    from dpfm_amd import _lib, ops
    x = torch.arange(10, dtype=torch.float32, device="cuda")
    assert float(ops.mean_f32(x)) == 4.5
    assert _lib.build_id() == _lib.tree_build_id()
