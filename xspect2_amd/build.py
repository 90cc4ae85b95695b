"""Build libxspect_hip.so in-tree for gfx950 with hipcc (no JIT, no cache dir)."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
SO_PATH = PKG / "libxspect_hip.so"
SOURCES = [CSRC / "xs_api.cpp", CSRC / "xs_fastx.cpp", CSRC / "xs_json.cpp", CSRC / "xs_kernels.hip"]
HEADERS = [CSRC / "xs_internal.h", ROOT / "include" / "xspect_hip.h"]
ARCH = os.environ.get("XSPECT2_AMD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libxspect_hip.so)")


def _stale() -> bool:
    if not SO_PATH.exists():
        return True
    t = SO_PATH.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS)


def build_library(force: bool = False, verbose: bool = False) -> Path:
    if not force and not _stale():
        return SO_PATH
    tmp = SO_PATH.with_suffix(".so.tmp")
    cmd = [hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared",
           "-Wno-pass-failed", "-Wno-unused-result", "-I", str(ROOT / "include"),
           "-o", str(tmp)] + [str(s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    env = dict(os.environ)
    env.setdefault("TMPDIR", "/tmp")
    res = subprocess.run(cmd, cwd=str(CSRC), capture_output=True, text=True, env=env)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, SO_PATH)
    return SO_PATH


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
