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
SOURCES = [CSRC / "xs_api.cpp", CSRC / "xs_fastx.cpp", CSRC / "xs_fastx_dev.hip", CSRC / "xs_json.cpp", CSRC / "xs_kernels.hip",
           CSRC / "xs_probe_fast.hip", CSRC / "xs_probe_wide.hip", CSRC / "xs_probe_slots.hip",
           CSRC / "xs_probe_general.hip", CSRC / "xs_probe_bloompart.hip",
           CSRC / "xs_probe_cobspart.hip"]
HEADERS = [CSRC / "xs_internal.h", CSRC / "xs_device.h", CSRC / "xs_part.h", ROOT / "include" / "xspect_hip.h"]
OBJ_DIR = PKG / "_build"
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
    """Compile each source to an object in parallel (the probe kernel families
    are separate translation units), then link the shared library."""
    if not force and not _stale():
        return SO_PATH
    from concurrent.futures import ThreadPoolExecutor

    OBJ_DIR.mkdir(exist_ok=True)
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wno-pass-failed",
             "-Wno-unused-result", "-I", str(ROOT / "include")]
    env = dict(os.environ)
    env.setdefault("TMPDIR", "/tmp")

    def run(cmd):
        if verbose:
            print(" ".join(cmd))
        res = subprocess.run(cmd, cwd=str(CSRC), capture_output=True, text=True, env=env)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")

    objs = [OBJ_DIR / (src.name + ".o") for src in SOURCES]
    newest_header = max(h.stat().st_mtime for h in HEADERS)

    def stale(src, obj):  # an object is rebuilt when its source or any header is newer
        return force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, newest_header)

    todo = [(src, obj) for src, obj in zip(SOURCES, objs) if stale(src, obj)]
    jobs = max(1, min(len(todo), os.cpu_count() or 1, 16))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(run, [[hipcc(), *flags, "-c", str(src), "-o", str(obj)] for src, obj in todo]))
    tmp = SO_PATH.with_suffix(".so.tmp")
    run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)])
    os.replace(tmp, SO_PATH)
    return SO_PATH


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
