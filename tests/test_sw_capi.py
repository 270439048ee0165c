"""CPU: the Smith-Waterman C ABI (include/hc_sw.h) is exported by the library,
the C++ drop-in header compiles, and without a GPU every entry point fails
loudly (no CPU fallback)."""
import os
import subprocess

import numpy as np
import pytest

import hcphmm
import hcsw
import sw_workloads as S


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(hcphmm.LIB_PATH):
        hcphmm.build()
    return hcsw.lib()


def test_exports_every_declared_sw_symbol(built):
    syms = hcsw.declared_symbols()
    assert len(syms) >= 7
    out = subprocess.run(["nm", "-D", "--defined-only", hcphmm.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert not [s for s in syms if s not in exported]


def test_sw_no_silent_fallback_without_gpu(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(hcsw.SWError) as e:
        hcsw.init()
    assert e.value.code == hcsw.ENODEV
    b = S.from_pairs([(b"ACGT", b"ACGA")])
    with pytest.raises(hcsw.SWError):
        hcsw.align_flat(b)


def test_sw_aligner_rejects_empty(built):
    with pytest.raises(ValueError):
        hcsw.SWAligner().align(b"", b"ACGT")
    with pytest.raises(ValueError):
        hcsw.SWAligner().align(b"ACGT", b"")


def test_sw_cpp_dropin_compiles(tmp_path):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "sw_dropin.cpp")], check=True)
