"""The C-ABI libraries load and export every symbol their headers declare
(CPU-only: no compute calls), and the GPU entry points fail loudly without a
GPU instead of falling back to the CPU."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header, prefix):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"\w+)\s*\(", txt)))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_hip_lib_exports_header(lz):
    names = declared("lz_hip.h", "lz_")
    assert len(names) >= 20
    syms = exported(lz.HIP_LIB)
    missing = [n for n in names if n not in syms]
    assert not missing, missing
    L = lz.hip_lib()  # loads without a GPU
    for n in names:
        assert hasattr(L, n)
    assert {n for n, _, _ in lz.HIP_SYMBOLS} == set(names), "python bindings out of sync with lz_hip.h"


def test_host_lib_exports_header(lz):
    names = declared("lz_host.h", "lzh_")
    syms = exported(lz.HOST_LIB)
    assert not [n for n in names if n not in syms]
    assert {n for n, _, _ in lz.HOST_SYMBOLS} == set(names), "python bindings out of sync with lz_host.h"


def test_hip_lib_is_gfx950_code_object(lz):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", lz.HIP_LIB], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(lz.HIP_LIB, "rb").read()
    assert b"gfx950" in blob


def test_no_silent_cpu_fallback(lz):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by -m gpu tests")
    L = lz.hip_lib()
    assert L.lz_device_ok(0) == 0
    h = ctypes.c_void_p()
    rc = L.lz_init(0, ctypes.byref(h))
    assert rc != 0 and L.lz_last_error()
    with pytest.raises(lz.LanczosError):
        lz.Handle(0)


def test_version_string(lz):
    assert b"gfx950" in lz.hip_lib().lz_version()
