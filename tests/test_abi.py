"""The C-ABI library loads and exports every symbol include/xspect_hip.h
declares (CPU only: no compute calls without a GPU)."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "xspect_hip.h"


def declared_functions() -> list[str]:
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(xs_[a-z0-9_]+)\s*\(", text)))


def test_header_parses_and_lists_entry_points():
    names = declared_functions()
    assert "xs_query" in names and "xs_bank_open" in names and "xs_query_device" in names
    assert len(names) >= 18


def test_library_exports_every_declared_symbol():
    from xspect2_amd import _lib
    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.SO_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (xs_[a-z0-9_]+)\b", out))
    for name in declared_functions():
        assert name in exported, f"{name} not exported"
        assert hasattr(lib, name)
    # the ctypes table covers the whole header
    assert set(_lib.SIGNATURES) == set(declared_functions())


def test_version_and_errors_without_gpu():
    from xspect2_amd import _lib
    lib = _lib.load()
    assert lib.xs_version() >= 100
    # argument errors are reported before any device work
    h = ctypes.c_void_p()
    rc = lib.xs_bank_open(b"/nonexistent/index.cobs_classic", 0, 0, ctypes.byref(h))
    assert rc == _lib.XS_ERR_IO
    assert b"cannot open" in lib.xs_last_error()
    rc = lib.xs_bank_open(b"/nonexistent", 7, 0, ctypes.byref(h))
    assert rc == _lib.XS_ERR_ARG


def test_product_does_not_import_oracle():
    """The product package never touches oracle/ (checker only)."""
    for py in (ROOT / "xspect2_amd").rglob("*.py"):
        src = py.read_text()
        assert "import oracle" not in src and "from oracle" not in src, py
        assert "liboracle" not in src, py
    for c in (ROOT / "xspect2_amd" / "csrc").iterdir():
        src = c.read_text()
        assert not re.search(r'#include\s+[<"][^>"]*oracle', src), c
        assert "xo_" not in re.sub(r"//.*", "", src), c


def test_no_environment_reads_on_the_query_path():
    """Path selection is a per-handle option (xs_bank_set_probe_options), not
    an environment variable read per call: the probe
    kernels' planners and the query code read no environment; what is left
    are the reader's two operational settings, each read once per process
    (function-local statics in xs_fastx.cpp)."""
    csrc = ROOT / "xspect2_amd" / "csrc"
    for f in sorted(csrc.glob("xs_probe_*.hip")) + [csrc / "xs_api.cpp", csrc / "xs_kernels.hip",
                                                     csrc / "xs_internal.h", csrc / "xs_json.cpp"]:
        assert "getenv" not in f.read_text(), f.name
    fx = (csrc / "xs_fastx.cpp").read_text()
    reads = re.findall(r'getenv\("([A-Z0-9_]+)"\)', fx)
    assert sorted(reads) == ["XSPECT2_AMD_FASTX_TRACE", "XSPECT2_AMD_FX_FIRST_MB", "XSPECT2_AMD_FX_RING"], reads
    for var in reads:  # each inside a static initialiser: read once
        i = fx.index(f'getenv("{var}")')
        assert "static" in fx[fx.rfind("\n", 0, fx.rfind("\n", 0, i)) - 200:i], var
