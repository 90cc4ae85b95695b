"""Build provenance (xspect2_amd/build.py): the library carries a build id,
a hash of its sources, headers, flags and target; build_library rebuilds when
the sources' id differs from the library's, not when file times change.

Runs on a copy of one source (xs_json.cpp, a host-only unit that compiles in
seconds) and the headers in a temporary directory, so the in-tree library is
untouched.  Needs hipcc (this container and the GPU box have it)."""
from __future__ import annotations

import os
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from xspect2_amd import build as B  # noqa: E402


def test_in_tree_library_matches_its_sources():
    """The shipped library was built from exactly the sources in the tree."""
    if not B.SO_PATH.exists():
        pytest.skip("library not built")
    assert B.so_build_id() == B.source_id()


def test_abi_reports_the_embedded_id():
    if not B.SO_PATH.exists():
        pytest.skip("library not built")
    from xspect2_amd import _lib
    assert _lib.build_id() == B.so_build_id() == B.source_id()


def test_rebuild_follows_content_not_mtime(tmp_path):
    try:
        B.hipcc()
    except RuntimeError:
        pytest.skip("hipcc not available")
    # the package layout: sources include "../../include/xspect_hip.h"
    csrc = tmp_path / "xspect2_amd" / "csrc"
    inc = tmp_path / "include"
    csrc.mkdir(parents=True)
    inc.mkdir()
    for h in B.HEADER_NAMES:
        shutil.copy(B.CSRC / h, csrc / h)
    shutil.copy(B.INCLUDE / "xspect_hip.h", inc / "xspect_hip.h")
    src = csrc / "xs_json.cpp"
    shutil.copy(B.CSRC / "xs_json.cpp", src)
    kw = dict(sources=[src], headers=[csrc / h for h in B.HEADER_NAMES] + [inc / "xspect_hip.h"],
              so_path=tmp_path / "lib.so", obj_dir=tmp_path / "_build")
    assert B.build_library(**kw) is True
    first = B.so_build_id(kw["so_path"])
    assert first == B.source_id(kw["sources"], kw["headers"])
    assert B.build_library(**kw) is False                      # same bytes: nothing to do
    st = src.stat()
    os.utime(src, (st.st_atime + 100, st.st_mtime + 100))     # touched, unchanged
    assert B.build_library(**kw) is False
    obj = kw["obj_dir"] / "xs_json.cpp.o"
    t_obj = obj.stat().st_mtime_ns
    src.write_bytes(src.read_bytes() + b"\n// one more byte\n")  # changed
    assert B.build_library(**kw) is True
    second = B.so_build_id(kw["so_path"])
    assert second != first and second == B.source_id(kw["sources"], kw["headers"])
    assert obj.stat().st_mtime_ns != t_obj                     # the changed unit was recompiled
