"""CPU-side checks of the C ABI: the library builds, loads, and exports every symbol include/ declares."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "faithdiff_hip.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^(?:int|long long|const char\*|void)\s+(fd_\w+)\(", txt, flags=re.M)))


def test_header_declares_expected_ops():
    syms = declared_symbols()
    for s in ["fd_gemm", "fd_flash_attn", "fd_group_norm", "fd_layer_norm", "fd_tlc_blend", "fd_tlc_cfg_euler_step"]:
        assert s in syms


def test_library_loads_and_exports_every_declared_symbol():
    from fdhip import lib
    so = lib.load()  # ctypes dlopen; no device call
    for s in declared_symbols():
        assert hasattr(so, s), s
    assert set(declared_symbols()) == set(lib.exported_symbols())
    assert lib.load().fd_version().decode().startswith("libfaithdiff_hip")


def test_library_is_gfx950_code_object():
    from fdhip import lib
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", lib.LIB_PATH], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-readelf unavailable")
    # the fat binary embeds a gfx950 code object bundle
    data = open(lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_ops_fail_loudly_without_gpu():
    import torch
    from fdhip import lib
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        lib.require_device()


def test_gemm_params_struct_matches_header():
    """ctypes layout of fd_gemm_params == C layout (field order from the header)."""
    from fdhip import lib
    txt = open(HDR).read()
    body = txt[txt.index("typedef struct fd_gemm_params"):txt.index("} fd_gemm_params;")]
    names = re.findall(r"(\w+)(?:,|;)", re.sub(r"/\*.*?\*/", "", body, flags=re.S))
    names = [n for n in names if n not in ("void", "int", "float", "long", "const")]
    assert [f[0] for f in lib.GemmParams._fields_] == names


def test_knob_table_defaults_and_no_environment_reads():
    """The planner knobs are one compiled-in table (csrc/knobs.hip + fdhip/knobs.py): set / restore through the C ABI,
    no getenv in the library, no FD_* environment read in the product's host code (only measurement scripts call
    knobs.apply_env)."""
    from fdhip import knobs
    from fdhip import lib
    assert knobs.changed() == {}
    with knobs.override(FD_GEMM256=0, FD_F8_KERNEL="dma", FD_LN_FOLD=0):
        assert knobs.changed() == {"FD_GEMM256": 0, "FD_F8_KERNEL": 1, "FD_LN_FOLD": 0}
    assert knobs.changed() == {}
    assert lib.load().fd_set_knob(b"FD_NO_SUCH_KNOB", 1, None) != 0
    assert knobs.apply_env({"FD_GEMM8_MIDK": "2", "UNRELATED": "1"}) == {"FD_GEMM8_MIDK": 2}
    lib.load().fd_reset_knobs()
    assert knobs.get("FD_GEMM8_MIDK") == knobs.default("FD_GEMM8_MIDK") == 3
    data = open(lib.LIB_PATH, "rb").read()
    assert b"getenv" not in data
    pkg = os.path.join(ROOT, "faithdiff-dev_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py") and f != "knobs.py":
                txt = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"environ(\.get)?[\[(]\s*[\"']FD_(?!LIB_PATH)", txt), f
