"""The C-ABI library loads and exports every symbol ``include/dkg.h`` declares.

CPU-only: no compute entry point is called with device data here; argument
validation paths that return before touching the GPU are exercised.
"""

import ctypes
import os
import re

import pytest

from dkg_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "dkg.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(dkg_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "dkg_forward" in names and "dkg_lines_kg" in names and len(names) >= 10


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"


def test_abi_version():
    assert _lib.load().dkg_abi_version() == _lib.ABI_VERSION


def test_frag_elems():
    lib = _lib.load()
    assert lib.dkg_frag_elems(1024, 256) == 1024 * 256
    assert lib.dkg_frag_elems(10, 10) == 16 * 16
    assert lib.dkg_frag_elems(0, 7) == 0


def test_struct_layout_matches_header():
    # int32 n, int32 kernel, 5 doubles, 6 pointers
    assert ctypes.sizeof(_lib.DkgOutput) == 4 + 4 + 5 * 8 + 6 * 8
    assert _lib.DkgOutput.inv_lengthscale.offset == 48


def test_validation_errors_without_device():
    lib = _lib.load()
    # no lines -> the reference's ValueError message (discretekg.py:466-470)
    st = lib.dkg_lines_kg(None, None, 3, 0, None, None, None)
    assert st == _lib.DKG_ERR_NO_LINES
    assert b"at least one line" in lib.dkg_last_error()
    with pytest.raises(ValueError, match="at least one line"):
        _lib.check(st, "dkg_lines_kg")
    # unsupported number of outputs
    outs = (_lib.DkgOutput * 1)()
    st = lib.dkg_forward(outs, 9, 2, None, 4, None, 1, None, 1, -1, None, None, None, 0, None)
    assert st == _lib.DKG_ERR_UNSUPPORTED
    # missing device state pointers -> argument error
    outs[0].n = 4
    outs[0].kernel = 2
    st = lib.dkg_forward(outs, 1, 2, None, 4, None, 1, None, 1, -1, None, None, None, 0, None)
    assert st == _lib.DKG_ERR_ARG
    # target out of range
    for f in ("inv_lengthscale", "train_x", "alpha", "root_frag", "disc_frag", "disc_mean"):
        setattr(outs[0], f, 16)
    st = lib.dkg_forward(outs, 1, 2, None, 4, None, 1, None, 1, 3, None, None, None, 0, None)
    assert st == _lib.DKG_ERR_ARG and b"target" in lib.dkg_last_error()
    # empty batch is a no-op
    assert lib.dkg_forward(outs, 1, 2, 16, 4, 16, 0, 16, 1, -1, 16, None, 16, 0, None) == _lib.DKG_OK
    # candidates in the kernel arguments: plan checks before any device work
    assert lib.dkg_plan_forward_grad_hostx(None, None, None, None, 1, None, None, None, None) == _lib.DKG_ERR_ARG
    blank = ctypes.create_string_buffer(lib.dkg_plan_bytes())  # a plan never initialised: no DKG_PLAN_GRAD
    st = lib.dkg_plan_forward_grad_hostx(blank, blank, None, None, 1, None, None, None, None)
    assert st == _lib.DKG_ERR_ARG and b"DKG_PLAN_GRAD" in lib.dkg_last_error()


def test_workspace_size_grows_with_problem():
    lib = _lib.load()
    outs = (_lib.DkgOutput * 2)()
    outs[0].n = outs[1].n = 256
    small = lib.dkg_forward_workspace(outs, 2, 256, 32, 8)
    big = lib.dkg_forward_workspace(outs, 2, 1024, 128, 16)
    assert 0 < small < big
    assert big >= 2 * 128 * 1024 * 8  # the covariance rows of both outputs


def test_prepare_output_validation_without_device():
    lib = _lib.load()
    assert lib.dkg_prepare_workspace(0) == 0
    assert lib.dkg_prepare_workspace(256) >= 256 * 256 * 8
    o = _lib.DkgOutput()
    o.n, o.kernel = 8, 2
    jit = ctypes.c_double(0.0)
    # NULL device pointers -> argument error before any device work
    assert lib.dkg_prepare_output(o, 2, None, 3, None, None, 0, None, None, ctypes.byref(jit), None) == _lib.DKG_ERR_ARG
    o.inv_lengthscale = o.train_x = 16
    args = (16, 3, 16, 16, lib.dkg_prepare_workspace(8), 16, 16, ctypes.byref(jit), None)
    o.n = 2000
    assert lib.dkg_prepare_output(o, 2, *args) == _lib.DKG_ERR_UNSUPPORTED
    o.n = 8
    assert lib.dkg_prepare_output(o, 17, *args) == _lib.DKG_ERR_UNSUPPORTED
    small = (16, 3, 16, 16, 8, 16, 16, ctypes.byref(jit), None)
    assert lib.dkg_prepare_output(o, 2, *small) == _lib.DKG_ERR_WORKSPACE
    from dkg_amd.errors import NotPSDError
    with pytest.raises(NotPSDError):
        _lib.check(_lib.DKG_ERR_NOT_PD, "dkg_prepare_output")


def test_f32_plan_flag_validation_without_device():
    """DKG_PLAN_F32 (include/dkg.h): its workspace holds the fp32 copies on top of the fp64 plan's,
    and it refuses the gradient flag before any device work."""
    lib = _lib.load()
    outs = (_lib.DkgOutput * 2)()
    for o in outs:
        o.n, o.kernel = 256, 2
        for f in ("inv_lengthscale", "train_x", "alpha", "root_frag", "disc_frag", "disc_mean"):
            setattr(o, f, 16)
    w64 = lib.dkg_plan_workspace(outs, 2, 2, 1024, 128, 16, 0)
    w32 = lib.dkg_plan_workspace(outs, 2, 2, 1024, 128, 16, _lib.DKG_PLAN_F32)
    # + per output: Q_X (128 x 256), R^T (256 x 256) and Q_D (1024 x 256) in fp32
    assert w32 - w64 >= 2 * 4 * (128 * 256 + 256 * 256 + 1024 * 256)
    host = ctypes.create_string_buffer(lib.dkg_plan_bytes())
    st = lib.dkg_plan_init(outs, 2, 2, 16, 1024, 16, 16, -1, 128, _lib.DKG_PLAN_F32 | _lib.DKG_PLAN_GRAD, 16,
                           1 << 40, host, 16, None)
    assert st == _lib.DKG_ERR_UNSUPPORTED and b"forward only" in lib.dkg_last_error()
    st = lib.dkg_plan_init(outs, 2, 2, 16, 1024, 16, 16, -1, 128, 64, 16, 1 << 40, host, 16, None)
    assert st == _lib.DKG_ERR_ARG and b"unknown plan flags" in lib.dkg_last_error()


def test_launcher_lifecycle_and_argument_checks():
    """dkg_launcher_*: worker threads start and stop, an empty launch set returns, bad arguments are refused
    (no graph is launched without a device)."""
    from dkg_amd.launch import GraphLauncher

    lib = _lib.load()
    L = GraphLauncher(3)
    L.arm(0.005)
    L.prepare("empty", [], [])
    L.launch("empty")
    offs = (ctypes.c_int * 2)(1, 0)  # decreasing offsets
    one = (ctypes.c_void_p * 1)(0)
    assert lib.dkg_launcher_graphs(L._h, 1, one, offs, one) == _lib.DKG_ERR_ARG
    L.close()
    h = ctypes.c_void_p()
    assert lib.dkg_launcher_create(0, ctypes.byref(h)) == _lib.DKG_ERR_ARG
