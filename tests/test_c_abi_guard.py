"""Every C-ABI entry point runs its body under xs::guard (xs_internal.h), so
no C++ exception unwinds into a ctypes caller (INTEGRATION.md §3 "Errors").
A source check: each exported function defined in the library's C++ units
either is a one-line accessor that cannot throw or opens with the guard."""
from __future__ import annotations

import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "xspect2_amd" / "csrc"
TRIVIAL = {"xs_version", "xs_last_error", "xs_fastx_close"}  # return a constant / a c_str / delete


def _definitions():
    for path in sorted(CSRC.glob("*.cpp")):
        lines = path.read_text().split("\n")
        for i, line in enumerate(lines):
            m = re.match(r"^[A-Za-z][\w\s\*]*?\b(xs_\w+)\(", line)
            if not m:
                continue
            j = i
            while not lines[j].rstrip().endswith(("{", ";")) and "{" not in lines[j]:
                j += 1
            if lines[j].rstrip().endswith(";"):
                continue  # a declaration
            yield path.name, m.group(1), line, lines[j + 1] if j + 1 < len(lines) else ""


def test_every_entry_point_is_guarded():
    header = (ROOT / "include" / "xspect_hip.h").read_text()
    declared = set(re.findall(r"\b(xs_\w+)\s*\(", header))
    seen, unguarded = set(), []
    for fname, name, line, first in _definitions():
        if name not in declared:
            continue
        seen.add(name)
        if name in TRIVIAL:
            assert line.rstrip().endswith("}"), f"{name} is no longer a one-liner: guard it"
            continue
        if "xs::guard(" not in first:
            unguarded.append(f"{fname}: {name}")
    assert not unguarded, unguarded
    # the generated build-id unit defines xs_build_id; everything else is defined here
    assert declared - seen <= {"xs_build_id"}, sorted(declared - seen)
