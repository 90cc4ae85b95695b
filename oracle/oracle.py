"""CPU ORACLE for the k-mer x filter probe path (test infrastructure only).

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module.  The product path (``xspect2_amd``)
never imports it and never falls back to it.

Two independent restatements live here and are checked against each other
and against golden vectors:

* ``liboracle.so`` (``xs_oracle.c``): plain C, OpenMP over reads.  Used for
  large cases and as the CPU baseline.
* pure-Python functions (suffix ``_py``): hash with the python-xxhash package
  (the same library XspecT imports at
  ``src/xspect/models/probabilistic_single_filter_model.py:11``).  Small cases
  only.

Parity status (see DESIGN.md "Oracle"):
* XXH64 / XXH3-64: pinned to python-xxhash 3.8.1 (tests/golden/xxh_vectors.json).
* k-mer positions and counts: pinned to the reference's known answers
  (``tests/test_probabilistic_filter_model.py:139-161`` -> 60 and 60/step).
* Scores/totals/SVM vector: pinned to the reference ``result.py`` run here
  (tests/golden/model_result_vectors.json).
* COBS index semantics and rbloom index generation: PARITY UNPINNED (the
  libraries are absent offline); this restatement follows their published
  algorithms as documented in xs_oracle.c.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
_LIB = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> Path:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    so = HERE / "liboracle.so"
    src = HERE / "xs_oracle.c"
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return so


def lib():
    global _LIB
    if _LIB is None:
        so = HERE / "liboracle.so"
        if not so.exists():
            build()
        L = ctypes.CDLL(str(so))
        L.xo_xxh64.restype = ctypes.c_uint64
        L.xo_xxh64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.xo_xxh3_64.restype = ctypes.c_uint64
        L.xo_xxh3_64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
        L.xo_cobs_signature_size.restype = ctypes.c_uint64
        L.xo_cobs_signature_size.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double]
        L.xo_canonical_cobs.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
        L.xo_canonical_bio.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
        L.xo_cobs_query.restype = ctypes.c_int
        L.xo_cobs_query.argtypes = [
            _u8p, _u64p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_uint32, ctypes.c_int, _u8p, _u64p, ctypes.c_uint64,
            ctypes.c_uint32, _u32p, _u64p, ctypes.c_int,
        ]
        L.xo_cobs_query_batched.restype = ctypes.c_int
        L.xo_cobs_query_batched.argtypes = L.xo_cobs_query.argtypes
        L.xo_xxh64_terms_check.restype = ctypes.c_uint64
        L.xo_xxh64_terms_check.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.xo_cobs_build.restype = ctypes.c_int
        L.xo_cobs_build.argtypes = [
            _u8p, _u64p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_uint32, ctypes.c_int, _u8p, _u64p, _u32p, ctypes.c_uint64,
        ]
        L.xo_bloom_indexes.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _u64p]
        L.xo_bloom_build.restype = ctypes.c_int
        L.xo_bloom_build.argtypes = [
            _u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, _u8p, _u64p, ctypes.c_uint64,
        ]
        L.xo_bloom_query.restype = ctypes.c_int
        L.xo_bloom_query.argtypes = [
            _u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, _u8p, _u64p,
            ctypes.c_uint64, ctypes.c_uint32, _u32p, _u64p, ctypes.c_int,
        ]
        L.xo_bloom_query_batched.restype = ctypes.c_int
        L.xo_bloom_query_batched.argtypes = L.xo_bloom_query.argtypes
        L.xo_num_threads.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


# ---------------------------------------------------------------- hashes
def xxh64(data: bytes, seed: int = 0) -> int:
    return int(lib().xo_xxh64(data, len(data), seed))


def xxh3_64(data: bytes) -> int:
    ok = ctypes.c_int(0)
    v = int(lib().xo_xxh3_64(data, len(data), ctypes.byref(ok)))
    if not ok.value:
        raise ValueError("xxh3 oracle supports inputs up to 240 bytes")
    return v


def signature_size(n: int, num_hashes: int, fpr: float) -> int:
    return int(lib().xo_cobs_signature_size(n, num_hashes, fpr))


def signature_size_py(n: int, num_hashes: int, fpr: float) -> int:
    return int(math.ceil(-num_hashes * n / math.log(1.0 - math.pow(fpr, 1.0 / num_hashes))))


# ---------------------------------------------------------------- canonical
def canonical_cobs(kmer: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(kmer))
    lib().xo_canonical_cobs(kmer, len(kmer), out)
    return out.raw


def canonical_bio(kmer: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(kmer))
    lib().xo_canonical_bio(kmer, len(kmer), out)
    return out.raw


_COBS_NORM = {ord(c): c for c in "ACGT"} | {ord(c): c.upper() for c in "acgt"}
_COBS_COMP = str.maketrans("ACGTN", "TGCAN")
_BIO_PAIRS = "ATTACGGCMKKMRYYRWWSSVBBVHDDHXXNN"
_BIO_COMP = str.maketrans(
    _BIO_PAIRS[0::2] + _BIO_PAIRS[0::2].lower(), _BIO_PAIRS[1::2] + _BIO_PAIRS[1::2].lower()
)


def canonical_cobs_py(kmer: str) -> str:
    fwd = "".join(_COBS_NORM.get(ord(c), "N") for c in kmer)
    rc = fwd.translate(_COBS_COMP)[::-1]
    return min(fwd, rc)


def canonical_bio_py(kmer: str) -> str:
    """min(kmer, str(kmer.reverse_complement())) as in
    probabilistic_single_filter_model.py:179 (Biopython IUPAC table)."""
    return min(kmer, kmer.translate(_BIO_COMP)[::-1])


def num_kmers(length: int, k: int, step: int = 1) -> int:
    """ceil((len(seq) - k + 1) / step)  (probabilistic_filter_model.py:462)."""
    return max(0, math.ceil((length - k + 1) / step))


# ---------------------------------------------------------------- packing
def pack(seqs) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate sequences (str/bytes) into (u8 buffer, u64 offsets[n+1])."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        offs[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8).copy()
    return buf, offs


# ---------------------------------------------------------------- COBS banks
class CobsBank:
    """Host image of a COBS classic (G=1, P=ceil(D/8)) or compact bank."""

    def __init__(self, rows: np.ndarray, sig: list[int], page: int, num_docs: int,
                 num_hashes: int, k: int):
        self.rows = np.ascontiguousarray(rows, dtype=np.uint8)
        self.sig = np.asarray(sig, dtype=np.uint64)
        self.P = int(page)
        self.D = int(num_docs)
        self.h = int(num_hashes)
        self.k = int(k)
        assert self.rows.size == int(self.sig.sum()) * self.P

    @classmethod
    def empty(cls, sig, page, num_docs, num_hashes, k):
        rows = np.zeros(int(np.sum(np.asarray(sig, dtype=np.uint64))) * page, dtype=np.uint8)
        return cls(rows, list(sig), page, num_docs, num_hashes, k)

    def build(self, seqs, docs) -> None:
        buf, offs = pack(seqs)
        d = np.ascontiguousarray(docs, dtype=np.uint32)
        rc = lib().xo_cobs_build(
            _p(self.rows, _u8p), _p(self.sig, _u64p), len(self.sig), self.P, self.D, self.h,
            self.k, _p(buf, _u8p), _p(offs, _u64p), _p(d, _u32p), len(d))
        if rc != 0:
            raise ValueError(f"xo_cobs_build failed ({rc})")

    def query_packed(self, buf, offs, step=1, threads=0):
        n = len(offs) - 1
        hits = np.zeros((n, self.D), dtype=np.uint32)
        nk = np.zeros(n, dtype=np.uint64)
        rc = lib().xo_cobs_query(
            _p(self.rows, _u8p), _p(self.sig, _u64p), len(self.sig), self.P, self.D, self.h,
            self.k, _p(buf, _u8p), _p(offs, _u64p), n, step, _p(hits, _u32p), _p(nk, _u64p),
            int(threads))
        if rc != 0:
            raise ValueError(f"xo_cobs_query failed ({rc})")
        return hits, nk

    def query(self, seqs, step=1, threads=0):
        buf, offs = pack(seqs)
        return self.query_packed(buf, offs, step, threads)

    def query_packed_batched(self, buf, offs, step=1, threads=0):
        """query_packed through xo_cobs_query_batched: the same answer,
        computed as a tuned CPU port would (bench.py's cpu_baseline)."""
        n = len(offs) - 1
        hits = np.zeros((n, self.D), dtype=np.uint32)
        nk = np.zeros(n, dtype=np.uint64)
        rc = lib().xo_cobs_query_batched(
            _p(self.rows, _u8p), _p(self.sig, _u64p), len(self.sig), self.P, self.D, self.h,
            self.k, _p(buf, _u8p), _p(offs, _u64p), n, step, _p(hits, _u32p), _p(nk, _u64p),
            int(threads))
        if rc != 0:
            raise ValueError(f"xo_cobs_query_batched failed ({rc})")
        return hits, nk

    # -- pure python (python-xxhash) restatement, small inputs only --------
    def query_py(self, seqs, step=1):
        import xxhash

        bases = np.concatenate([[0], np.cumsum(self.sig.astype(np.int64) * self.P)])
        out = []
        for s in seqs:
            s = s.decode() if isinstance(s, bytes) else s
            counts = [0] * self.D
            for i in range(num_kmers(len(s), self.k, step)):
                c = canonical_cobs_py(s[i * step:i * step + self.k]).encode()
                hs = [xxhash.xxh64_intdigest(c, seed=j) for j in range(self.h)]
                for d in range(self.D):
                    g, bit = divmod(d, 8 * self.P)
                    ok = True
                    for hv in hs:
                        row = int(bases[g]) + (hv % int(self.sig[g])) * self.P
                        if not (self.rows[row + (bit >> 3)] >> (bit & 7)) & 1:
                            ok = False
                            break
                    counts[d] += ok
            out.append(counts)
        return np.asarray(out, dtype=np.uint32).reshape(len(out), self.D)


# ---------------------------------------------------------------- rbloom
class BloomFilter:
    """Host image of an rbloom filter (UNVERIFIED index generator)."""

    def __init__(self, bits: np.ndarray, num_hashes: int, k: int):
        self.bits = np.ascontiguousarray(bits, dtype=np.uint8)
        self.K = int(num_hashes)
        self.k = int(k)

    @staticmethod
    def params(expected_items: int, fpr: float) -> tuple[int, int]:
        """(nbytes, num_hashes) for Bloom(expected_items, fpr) (restated)."""
        size_bits = int(-expected_items * math.log(fpr) / (math.log(2) ** 2))
        nh = max(1, math.ceil(size_bits / expected_items * math.log(2)))
        return (size_bits + 7) // 8, nh

    def build(self, seqs) -> None:
        buf, offs = pack(seqs)
        rc = lib().xo_bloom_build(_p(self.bits, _u8p), self.bits.size, self.K, self.k,
                                  _p(buf, _u8p), _p(offs, _u64p), len(offs) - 1)
        if rc != 0:
            raise ValueError(f"xo_bloom_build failed ({rc})")

    def query_packed(self, buf, offs, step=1, threads=0):
        n = len(offs) - 1
        hits = np.zeros(n, dtype=np.uint32)
        nk = np.zeros(n, dtype=np.uint64)
        rc = lib().xo_bloom_query(_p(self.bits, _u8p), self.bits.size, self.K, self.k,
                                  _p(buf, _u8p), _p(offs, _u64p), n, step, _p(hits, _u32p),
                                  _p(nk, _u64p), int(threads))
        if rc != 0:
            raise ValueError(f"xo_bloom_query failed ({rc})")
        return hits, nk

    def query_packed_batched(self, buf, offs, step=1, threads=0):
        """query_packed through xo_bloom_query_batched: the same answer,
        computed as a tuned CPU port would (bench.py's cpu_baseline)."""
        n = len(offs) - 1
        hits = np.zeros(n, dtype=np.uint32)
        nk = np.zeros(n, dtype=np.uint64)
        rc = lib().xo_bloom_query_batched(_p(self.bits, _u8p), self.bits.size, self.K, self.k,
                                          _p(buf, _u8p), _p(offs, _u64p), n, step, _p(hits, _u32p),
                                          _p(nk, _u64p), int(threads))
        if rc != 0:
            raise ValueError(f"xo_bloom_query_batched failed ({rc})")
        return hits, nk

    def query(self, seqs, step=1, threads=0):
        buf, offs = pack(seqs)
        return self.query_packed(buf, offs, step, threads)

    def indexes(self, h: int) -> list[int]:
        out = np.zeros(self.K, dtype=np.uint64)
        lib().xo_bloom_indexes(h, self.K, self.bits.size * 8, _p(out, _u64p))
        return [int(x) for x in out]

    def contains_py(self, kmer: str) -> bool:
        import xxhash

        h = xxhash.xxh3_64_intdigest(canonical_bio_py(kmer).encode())
        m = self.bits.size * 8
        st = h
        M = (0x2360ED051FC65DA4 << 64) | 0x4385DF649FCCF645
        C = (0x5851F42D4C957F2D << 64) | 0x14057B7EF767814F
        for _ in range(self.K):
            st = (st * M + C) & ((1 << 128) - 1)
            idx = (st >> 64) % m
            if not (int(self.bits[idx >> 3]) >> (idx & 7)) & 1:
                return False
        return True


# ---------------------------------------------------------------- MLST
def sequence_splitter(seq: str, allele_len: int, k: int) -> list[str]:
    """Restates probabilistic_filter_mlst_model.py:382-426."""
    n = len(seq)
    if n < 1_000_000:
        width = allele_len
    elif n < 10_000_000:
        width = allele_len * 10
    else:
        width = allele_len * 100
    parts, start = [], 0
    while start + width <= n:
        parts.append(seq[start:start + width])
        start += width - k + 1
    if start < n:
        tail = seq[start:]
        if len(tail) < k:
            parts[-1] += tail
        else:
            parts.append(tail)
    return parts


def num_threads() -> int:
    return int(lib().xo_num_threads())


if __name__ == "__main__":  # pragma: no cover
    print(build(), os.cpu_count())


# ---------------------------------------------------------------- file layouts (spec)
def cobs_classic_file(names: list[str], k: int, h: int, sig: int, rows: np.ndarray) -> bytes:
    """COBS classic index file as restated (UNVERIFIED, from recollection of
    cobs-reloaded): "COBS:CLASSIC_INDEX", u32 version 1, u32 num_docs, u32
    term_size, u8 canonicalize = 1, u64 signature_size, u64 num_hashes, the
    doc names each ending in '\\n', "CLASSIC_INDEX", then the S x ceil(D/8)
    row-major payload (doc d = byte d >> 3, bit d & 7)."""
    import struct
    head = b"COBS:CLASSIC_INDEX" + struct.pack("<IIIBQQ", 1, len(names), k, 1, sig, h)
    head += b"".join(n.encode() + b"\n" for n in names) + b"CLASSIC_INDEX"
    return head + np.ascontiguousarray(rows, dtype=np.uint8).tobytes()


def cobs_compact_file(names: list[str], k: int, h: int, sig: list[int], page: int, rows: np.ndarray) -> bytes:
    """COBS compact index file as restated (UNVERIFIED): "COBS:COMPACT_INDEX",
    u32 version 1, u32 term_size, u8 canonicalize = 1, u64 num_groups, per group
    (u64 signature_size, u64 num_hashes), u64 page_size, u32 num_docs, names,
    "COMPACT_INDEX", zero padding to a multiple of page_size, then each group's
    signature_size rows of page_size bytes."""
    import struct
    head = b"COBS:COMPACT_INDEX" + struct.pack("<IIBQ", 1, k, 1, len(sig))
    head += b"".join(struct.pack("<QQ", s, h) for s in sig) + struct.pack("<QI", page, len(names))
    head += b"".join(n.encode() + b"\n" for n in names) + b"COMPACT_INDEX"
    head += b"\0" * ((page - len(head) % page) % page)
    return head + np.ascontiguousarray(rows, dtype=np.uint8).tobytes()


def rbloom_file(num_hashes: int, bits: np.ndarray) -> bytes:
    """rbloom filter file as restated (UNVERIFIED): u64 little-endian K, then
    the filter bytes (bit i = byte i >> 3, bit i & 7)."""
    import struct
    return struct.pack("<Q", num_hashes) + np.ascontiguousarray(bits, dtype=np.uint8).tobytes()


def bloom_indexes_py(hash64: int, nhash: int, mbits: int) -> list[int]:
    """rbloom's K bit indices as restated (UNVERIFIED): a 128-bit LCG
    state <- state * M + C mod 2^128 from state = the XXH3-64 hash, index =
    (state >> 64) mod m, K times (Python big integers)."""
    M = (0x2360ED051FC65DA4 << 64) | 0x4385DF649FCCF645
    C = (0x5851F42D4C957F2D << 64) | 0x14057B7EF767814F
    st, out = hash64, []
    for _ in range(nhash):
        st = (st * M + C) % (1 << 128)
        out.append((st >> 64) % mbits)
    return out
