"""Build libxspect_hip.so in-tree for gfx950 with hipcc (no JIT, no cache dir).

Provenance is by content, not by file times: the library carries a build id,
the first 16 hex digits of a SHA-256 over the sources, headers, flags and
target (``source_id``), embedded as a tagged string (``xs_build_id()`` in the
ABI) and read back from the file without loading it (``so_build_id``).
``build_library`` rebuilds when the two differ, and each object when the hash
of its source + the headers + the flags differs from the stamp beside it; a
touched file with unchanged bytes rebuilds nothing.
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
SO_PATH = PKG / "libxspect_hip.so"
SOURCE_NAMES = ["xs_api.cpp", "xs_pool.cpp", "xs_fastx.cpp", "xs_fastx_dev.hip", "xs_json.cpp", "xs_kernels.hip",
                "xs_probe_fast.hip", "xs_probe_vslice.hip", "xs_probe_wide.hip", "xs_probe_slots.hip", "xs_probe_general.hip",
                "xs_probe_bloompart.hip", "xs_probe_cobspart.hip"]
HEADER_NAMES = ["xs_internal.h", "xs_device.h", "xs_part.h"]
SOURCES = [CSRC / s for s in SOURCE_NAMES]
HEADERS = [CSRC / h for h in HEADER_NAMES] + [INCLUDE / "xspect_hip.h"]
OBJ_DIR = PKG / "_build"
ARCH = "gfx950"  # MI355X only: the kernels use gfx950 instructions (LDS-DMA dwordx4, v_bitop3)
ID_TAG = b"xspect2-build-id:"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libxspect_hip.so)")


def _flags() -> list[str]:
    return ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wno-pass-failed", "-Wno-unused-result"]


def _digest(parts) -> str:
    h = hashlib.sha256()
    for name, data in parts:
        h.update(name.encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    return h.hexdigest()[:16]


def source_id(sources=None, headers=None) -> str:
    """Build id of the library these sources, headers, flags and target make."""
    sources = SOURCES if sources is None else sources
    headers = HEADERS if headers is None else headers
    return _digest([("flags", " ".join(_flags()).encode())] +
                   [(p.name, p.read_bytes()) for p in sorted(sources + headers, key=lambda p: p.name)])


def so_build_id(so_path: Path = SO_PATH) -> str | None:
    """The id embedded in a built library (None: missing file or no tag)."""
    try:
        data = Path(so_path).read_bytes()
    except OSError:
        return None
    m = re.search(re.escape(ID_TAG) + rb"([0-9a-f]{16})\0", data)
    return m.group(1).decode() if m else None


def build_library(force: bool = False, verbose: bool = False, sources=None, headers=None,
                  so_path: Path = SO_PATH, obj_dir: Path = OBJ_DIR) -> bool:
    """Compile each source to an object in parallel (the probe kernel families
    are separate translation units), then link the shared library with the
    build-id unit.  Returns True when the library was (re)built."""
    sources = SOURCES if sources is None else sources
    headers = HEADERS if headers is None else headers
    want = source_id(sources, headers)
    if not force and so_build_id(so_path) == want:
        return False
    from concurrent.futures import ThreadPoolExecutor

    obj_dir.mkdir(parents=True, exist_ok=True)
    inc = sorted({str(h.parent) for h in headers})
    flags = _flags() + [x for d in inc for x in ("-I", d)]
    env = dict(os.environ)
    env.setdefault("TMPDIR", "/tmp")

    def run(cmd, cwd):
        if verbose:
            print(" ".join(cmd))
        res = subprocess.run(cmd, cwd=str(cwd), capture_output=True, text=True, env=env)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")

    head = [(h.name, h.read_bytes()) for h in sorted(headers, key=lambda p: p.name)]
    objs = [obj_dir / (src.name + ".o") for src in sources]
    todo = []
    for src, obj in zip(sources, objs):
        key = _digest([("flags", " ".join(flags).encode()), (src.name, src.read_bytes())] + head)
        stamp = obj.with_name(obj.name + ".id")
        if force or not obj.exists() or not stamp.exists() or stamp.read_text().strip() != key:
            todo.append((src, obj, stamp, key))
    # the id unit: one tagged string and xs_build_id() (include/xspect_hip.h)
    id_src = obj_dir / "xs_build_id.cpp"
    id_src.write_text(f'extern "C" {{\n__attribute__((used)) const char xs_build_id_tag[] = '
                      f'"{ID_TAG.decode()}{want}";\n'
                      f'const char* xs_build_id(void) {{ return xs_build_id_tag + {len(ID_TAG)}; }}\n}}\n')
    id_obj = obj_dir / "xs_build_id.o"

    def compile_one(job):
        src, obj, stamp, key = job
        run([hipcc(), *flags, "-c", str(src), "-o", str(obj)], src.parent)
        stamp.write_text(key + "\n")

    jobs = max(1, min(len(todo) + 1, os.cpu_count() or 1, 16))
    with ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(compile_one, j) for j in todo]
        futs.append(ex.submit(run, [hipcc(), "-O2", "-fPIC", "-c", str(id_src), "-o", str(id_obj)], obj_dir))
        for f in futs:
            f.result()
    tmp = Path(str(so_path) + ".tmp")
    run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs), str(id_obj)],
        obj_dir)
    os.replace(tmp, so_path)
    if so_build_id(so_path) != want:
        raise RuntimeError(f"{so_path}: build id not found after linking")
    return True


if __name__ == "__main__":
    print(build_library(force=True, verbose=True), so_build_id())
