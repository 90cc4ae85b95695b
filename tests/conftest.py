"""pytest configuration: the `gpu` marker and shared fixtures.

CPU runs: ``pytest -m "not gpu"`` (oracle vs golden vectors, host logic, ABI
exports, gloo multi-process).  GPU runs: ``pytest -m gpu`` (parity of the HIP
path against the oracle through the C ABI).  GPU tests never skip silently:
a missing extension or device is a failure.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = Path(__file__).resolve().parent / "golden"
for p in (str(ROOT), str(ROOT / "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def golden():
    def _load(name: str):
        return json.loads((GOLDEN / name).read_text())
    return _load


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # test infrastructure only
    oracle.build()
    return oracle
