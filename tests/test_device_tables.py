"""Byte-table tricks of the device k-mer assembly, checked exhaustively on the
CPU against the plain predicates they replace (xspect2_amd/csrc/xs_device.h).

The constants are read from the shipped header, and v_perm_b32 is restated
from the CDNA4 ISA (each result byte is byte `sel` of the 64-bit value
{S0:S1} for selector bytes 0..7).  The device code masks every selector to
0..7 (`& 0x07070707`), so the special selectors (>= 8) cannot occur and are
not modelled.  A wrong constant would not always show in the GPU parity
tests: the genus path falls back to a per-byte table when a window fails the
A/C/G/T/N test, and that fallback gives the same answer, so only these tests
pin the fast-path predicate itself.
"""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np

HDR = Path(__file__).resolve().parents[1] / "xspect2_amd" / "csrc" / "xs_device.h"
M32 = np.uint32(0xFFFFFFFF)


def _body(name: str) -> str:
    src = HDR.read_text()
    i = src.index(f" {name}(")
    return src[i:src.index("\n}", i)]


def _perm_consts(name: str, arg: str) -> tuple[int, int]:
    m = re.search(r"__builtin_amdgcn_perm\((0x[0-9A-Fa-f]+)u,\s*(0x[0-9A-Fa-f]+)u,\s*" + arg + r" & 0x07070707u\)",
                  _body(name))
    assert m, f"{name}: perm call not found"
    return int(m.group(1), 16), int(m.group(2), 16)


def v_perm(s0: int, s1: int, sel: np.ndarray) -> np.ndarray:
    """v_perm_b32 with every selector byte in 0..7."""
    table = np.frombuffer(((s0 << 32) | s1).to_bytes(8, "little"), dtype=np.uint8)
    sel = sel.astype(np.uint32)
    out = np.zeros_like(sel)
    for lane in range(4):
        b = (sel >> np.uint32(8 * lane)) & np.uint32(0xFF)
        assert int(b.max()) < 8
        out |= table[b].astype(np.uint32) << np.uint32(8 * lane)
    return out


def zero_bytes(v: np.ndarray) -> np.ndarray:
    v = v.astype(np.uint32)
    return ~(((v & np.uint32(0x7F7F7F7F)) + np.uint32(0x7F7F7F7F)) | v | np.uint32(0x7F7F7F7F)) & M32


def bytes_equal(x: np.ndarray, c: int) -> np.ndarray:
    return zero_bytes(x ^ np.uint32(c * 0x01010101))


def _words() -> np.ndarray:
    """Every byte value in every lane (others random), plus 2^22 random words
    and words drawn from the bytes that matter (ACGTN, both cases, 0, 0xFF)."""
    rng = np.random.default_rng(0)
    parts = []
    for lane in range(4):
        base = rng.integers(0, 1 << 32, 256 * 16, dtype=np.uint64).astype(np.uint32)
        vals = np.tile(np.arange(256, dtype=np.uint32), 16)
        mask = np.uint32(0xFF << (8 * lane))
        parts.append((base & ~mask) | (vals << np.uint32(8 * lane)))
    parts.append(rng.integers(0, 1 << 32, 1 << 22, dtype=np.uint64).astype(np.uint32))
    hot = np.frombuffer(b"ACGTNacgtnRY\x00\xff\x41\x43", dtype=np.uint8)
    parts.append(hot[rng.integers(0, hot.size, (1 << 20, 4))].view("<u4").reshape(-1).astype(np.uint32))
    return np.concatenate(parts)


def _lanes(x: np.ndarray) -> np.ndarray:
    return x.view(np.uint8).reshape(-1, 4)  # little endian: column = byte lane


def test_acgtn_bytes_equals_five_byte_compares():
    s0, s1 = _perm_consts("acgtn_bytes", "x")
    x = _words()
    got = zero_bytes(v_perm(s0, s1, x & np.uint32(0x07070707)) ^ x)
    want = np.zeros_like(x)
    for c in b"ACGTN":
        want |= bytes_equal(x, c)
    assert np.array_equal(got, want)
    # and the compares themselves are the plain per-byte predicate
    is_acgtn = np.isin(_lanes(x), np.frombuffer(b"ACGTN", dtype=np.uint8))
    assert np.array_equal(_lanes(want) == 0x80, is_acgtn)
    assert set(np.unique(_lanes(want)).tolist()) <= {0, 0x80}


def test_comp4_complements_acgtn_and_zero():
    s0, s1 = _perm_consts("comp4", "f")
    comp = {ord("A"): ord("T"), ord("C"): ord("G"), ord("G"): ord("C"), ord("T"): ord("A"),
            ord("N"): ord("N"), 0: 0}
    keys = np.array(sorted(comp), dtype=np.uint8)
    rng = np.random.default_rng(1)
    f = keys[rng.integers(0, keys.size, (1 << 18, 4))]
    f = np.concatenate([f, np.stack(np.meshgrid(keys, keys, keys, keys), -1).reshape(-1, 4)])
    words = np.ascontiguousarray(f).view("<u4").reshape(-1).astype(np.uint32)
    got = _lanes(v_perm(s0, s1, words & np.uint32(0x07070707)))
    want = np.vectorize(comp.get)(f).astype(np.uint8)
    assert np.array_equal(got, want)


def test_acgt_bytes_equals_four_byte_compares():
    s0, s1 = _perm_consts("acgt_bytes", "u")
    x = _words()
    got = zero_bytes(v_perm(s0, s1, x & np.uint32(0x07070707)) ^ x)
    want = np.zeros_like(x)
    for c in b"ACGT":
        want |= bytes_equal(x, c)
    assert np.array_equal(got, want)
    assert np.array_equal(_lanes(want) == 0x80, np.isin(_lanes(x), np.frombuffer(b"ACGT", dtype=np.uint8)))


def test_cobs_norm4_equals_per_byte_normalisation():
    body = _body("cobs_norm4")
    assert "x & 0xDFDFDFDFu" in body and "acgt_bytes(u)" in body and "0x4E4E4E4Eu" in body
    s0, s1 = _perm_consts("acgt_bytes", "u")
    x = _words()
    u = x & np.uint32(0xDFDFDFDF)
    ok = zero_bytes(v_perm(s0, s1, u & np.uint32(0x07070707)) ^ u)
    m = ((ok >> np.uint32(7)) * np.uint32(0xFF)) & M32
    got = _lanes((u & m) | (np.uint32(0x4E4E4E4E) & ~m & M32))
    b = _lanes(x)
    up = np.where((b >= ord("a")) & (b <= ord("z")), b - 32, b).astype(np.uint8)
    want = np.where(np.isin(up, np.frombuffer(b"ACGT", dtype=np.uint8)), up, ord("N")).astype(np.uint8)
    assert np.array_equal(got, want)
