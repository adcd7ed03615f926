"""CPU: the C-ABI library loads, exports every symbol include/clonos_engine.h declares,
and fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "clonos_engine.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(clg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from clonos_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(_lib.EXPORTED) == names


def test_abi_version_and_struct_sizes():
    from clonos_amd import _lib
    assert _lib.lib.clg_abi_version() == 6
    assert ctypes.sizeof(_lib.IflReplayRes) == 48
    assert ctypes.sizeof(_lib.IflReplayReq) == 24
    assert ctypes.sizeof(_lib.CausalLogIdC) == 24
    assert ctypes.sizeof(_lib.Config) == 32
    assert ctypes.sizeof(_lib.SliceReq) == 32
    assert ctypes.sizeof(_lib.SliceRes) == 24
    assert ctypes.sizeof(_lib.DeltaReq) == 32
    assert ctypes.sizeof(_lib.Decoded) == 136
    assert ctypes.sizeof(_lib.KernelStat) == 56
    hdr = open(os.path.join(ROOT, "include", "clonos_engine.h")).read()
    assert re.search(r"#define CLG_DECODE_MAX_INFLIGHT (\d+)", hdr).group(1) == str(_lib.CLG_DECODE_MAX_INFLIGHT)


def test_kernels_built_for_gfx950():
    from clonos_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    for k in (b"k_dec_tables", b"k_dec_emit", b"k_gather", b"k_scatter", b"k_dec_resolve"):
        assert k in blob


def test_no_cpu_fallback_without_gpu(have_gpu):
    if have_gpu:
        pytest.skip("GPU present")
    from clonos_amd import ClonosError, Engine
    with pytest.raises(ClonosError) as ex:
        Engine()
    assert ex.value.status == -13  # CLG_E_DEVICE


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "clonos_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f), errors="replace").read()
                for pat in (r"import\s+.*oracle", r"from\s+\S*oracle", r"liboracle", r"\borc_[a-z]", r"pyref"):
                    assert not re.search(pat, txt), (f, pat)
