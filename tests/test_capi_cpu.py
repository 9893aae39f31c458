"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/niti_hip.h
declares, and its host-only entry points validate arguments (no device calls here)."""
import ctypes as C
import subprocess

import pytest


@pytest.fixture(scope="module")
def L():
    from niti_amd import _lib
    return _lib


def test_library_loads_and_reports_version(L):
    assert b"gfx950" in L.lib().niti_version()


def test_every_header_symbol_is_exported(L):
    names = L.header_functions()
    assert len(names) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:  # and ctypes resolves them
        getattr(L.lib(), n)


def test_code_object_targets_gfx950(L):
    data = open(L.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_create_execution_validation(L):
    lib = L.lib()
    h = C.c_void_p()
    c = L.ConvCommon()
    c.kernel_x = c.kernel_y = 3
    c.stride_x = c.stride_y = c.dilate_x = c.dilate_y = 1
    c.group = 1
    assert lib.niti_create_execution(999, C.byref(c), C.byref(h)) == 2      # NOT_SUPPORT
    assert lib.niti_create_execution(700, None, C.byref(h)) == 5            # INVALID_VALUE
    c.group = 2
    assert lib.niti_create_execution(700, C.byref(c), C.byref(h)) == 2      # grouped conv: NOT_SUPPORT
    c.group = 1
    for op in (700, 701, 705, 706, 714, 715, 718, 800, 802, 807, 810, 811, 812, 814, 815, 818, 819, 820, 821, 822):
        assert lib.niti_create_execution(op, C.byref(c), C.byref(h)) == 0
        assert lib.niti_execution_workspace_bytes(h) == 0
        lib.niti_destroy_execution(h)
    for op in (703, 704, 711, 713, 801, 803, 804, 805, 808, 809, 813, 817):  # no parameters: common may be NULL
        assert lib.niti_create_execution(op, None, C.byref(h)) == 0
        lib.niti_destroy_execution(h)


def test_geometry(L):
    lib = L.lib()
    g = L.Geom(256, 3, 32, 32, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0)
    assert lib.niti_geom_finalize(C.byref(g)) == 0
    assert (g.oh, g.ow, g.cip, g.cop, g.np) == (32, 32, 16, 64, 256)
    g = L.Geom(5, 20, 12, 12, 52, 5, 5, 1, 1, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0)
    assert lib.niti_geom_finalize(C.byref(g)) == 0
    assert (g.oh, g.ow, g.cip, g.cop, g.np) == (8, 8, 32, 64, 16)
    g = L.Geom(1, 1, 2, 2, 1, 5, 5, 1, 1, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0)
    assert lib.niti_geom_finalize(C.byref(g)) == 3  # COMPUTE_SIZE_ERROR


def test_row_conv_speculative_modes_validation(L):
    """Modes 3 / 4 (the speculative pair) need the state buffer that holds the layer's hint slot;
    modes past 4 are refused; the slot accessor is pure pointer arithmetic (no device access)."""
    lib = L.lib()
    g = L.Geom(2, 64, 56, 56, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0)
    assert lib.niti_geom_finalize(C.byref(g)) == 0
    dummy = C.c_void_p(16)  # never dereferenced: the calls fail validation first
    for mode in (3, 4):
        assert lib.niti_conv_fwd_rows(C.byref(g), dummy, dummy, None, None, None, 0, dummy, None, None, mode, dummy,
                                      None, 0, None, None) == 5  # INVALID_VALUE: no state
        assert lib.niti_conv_dgrad_rows(C.byref(g), dummy, dummy, None, None, None, 0, dummy, None, None, None,
                                        None, None, mode, dummy, None, 0, None, None) == 5
    assert lib.niti_conv_fwd_rows(C.byref(g), dummy, dummy, None, None, None, 0, dummy, None, None, 5, dummy, dummy, 0,
                                  None, None) == 5
    base = 4096
    fwd, dg = lib.niti_rows_spec_slot(C.c_void_p(base), 0), lib.niti_rows_spec_slot(C.c_void_p(base), 1)
    assert fwd is not None and dg is not None and dg - fwd == 128  # one 128-byte line per direction
    assert (fwd - base) // 4 + 5 <= 1216  # inside NITI_ROWCONV_STATE_WORDS
    assert lib.niti_rows_spec_slot(None, 0) is None


def test_no_fallback_when_library_missing(tmp_path, monkeypatch):
    import importlib

    from niti_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError):
        _lib.lib()
    importlib.reload(_lib)


@pytest.mark.parametrize("unit", ["niti_wgrad", "niti_kernels", "niti_rowconv"])
def test_asm_ring_kernels_no_inflight_register_reuse(tmp_path, unit):
    """Kernels with inline-asm load rings count their own waits (hipcc does not know when such a
    load lands): no instruction may touch a register such a load is still writing.  Compiles the
    translation unit to gfx950 assembly and scans every asm-ring kernel in it (the P16 weight
    gradient's buffer_load ring; the GEMM, tap-sharing and first-layer kernels' ds_read fragment
    rings) with tools/isa_inflight.py."""
    import os
    import shutil
    import subprocess
    import sys
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "mandheling-dsp-training_amd", "csrc", unit + ".hip")
    asm = tmp_path / (unit + ".s")
    subprocess.run([hipcc, "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++20", "-S", src, "-o",
                    str(asm)], check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "isa_inflight.py"), str(asm)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert " 0 asm-ring kernels" not in r.stdout, r.stdout


def test_execution_status_plumbing(L):
    """The error-status entry point without a device: a NULL handle is INVALID_VALUE, and an
    Execution whose launches carry no error word (not resized, so no fused row path) reports
    NO_ERROR without touching the GPU.  The forced-timeout path is tests/test_gpu_exec_host.py."""
    lib = L.lib()
    assert lib.niti_execution_status(None, None) == 5
    h = C.c_void_p()
    c = lib.niti_create_execution.argtypes[1]._type_()  # the ConvCommon class the loaded library binds
    c.kernel_x = c.kernel_y = 3
    c.stride_x = c.stride_y = c.dilate_x = c.dilate_y = 1
    c.pad_x = c.pad_y = 1
    c.group = 1
    for op in (700, 701, 715):
        assert lib.niti_create_execution(op, C.byref(c), C.byref(h)) == 0
        assert lib.niti_execution_status(h, None) == 0
        lib.niti_destroy_execution(h)
    lib.niti_diag_rowconv_barrier(0, 0)  # host-side setter: no device call
