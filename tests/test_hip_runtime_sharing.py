"""One HIP runtime per process (xspect2_amd._lib._preload_hip_runtime).

torch's ROCm wheel carries its own libamdhip64; loading this library first
without care puts /opt/rocm's runtime and torch's side by side in a process
that later imports torch, and device pointers then do not pass between them.
The library now loads torch's runtime itself (not torch: importing it cost a
one-shot classify process 1.2 s).  Runs on the CPU: loading needs no GPU."""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import json, sys
sys.path.insert(0, %r)
from xspect2_amd import _lib
_lib.load()
loaded_torch = "torch" in sys.modules
import torch  # noqa: F401
maps = open("/proc/self/maps").read().split("\n")
hip = sorted({l.split()[-1] for l in maps if "libamdhip64" in l})
hsa = sorted({l.split()[-1] for l in maps if "libhsa-runtime64" in l})
print(json.dumps({"torch_imported_by_load": loaded_torch, "hip": hip, "hsa": hsa}))
"""


def test_library_load_does_not_import_torch_and_shares_its_runtime():
    pytest.importorskip("torch")
    r = subprocess.run([sys.executable, "-c", CHILD % str(ROOT)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert not got["torch_imported_by_load"]
    assert len(got["hip"]) == 1, got["hip"]  # one libamdhip64 mapped, torch's
    assert "torch" in got["hip"][0]
    assert len(got["hsa"]) <= 1, got["hsa"]
