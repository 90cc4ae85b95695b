"""Native FASTA/FASTQ reader (xs_fastx_*) against the pure-Python restatement
of Biopython's parsers (oracle/fastx.py).  CPU only: the reader is host code.

Files are generated with the edge cases Bio.SeqIO meets in practice: text
before the first record, empty records, wrapped lines, CRLF, spaces and tabs
inside sequence lines, headers without descriptions, blank lines between FASTQ
records, '@' and '+' as quality characters, and files large enough that one
batch is split over many threads.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import fastx as ofx  # noqa: E402  (test-only checker)

from xspect2_amd.file_io import FastxReader, get_record_iterator, read_batches  # noqa: E402


def _pick(rng, alphabet: bytes, n: int) -> bytes:
    return rng.choice(np.frombuffer(alphabet, dtype=np.uint8), n).tobytes()


def _fasta_text(rng, n, wrap=True, crlf=False, junk=True) -> bytes:
    out = [b"; leading text the parser skips\n"] if junk else []
    nl = b"\r\n" if crlf else b"\n"
    for i in range(n):
        L = int(rng.integers(0, 400))
        seq = _pick(rng, b"ACGTNacgtn", L)
        desc = [b"", b" some description", b"\tdesc with tab", b"   "][i % 4]
        out.append(b">read_%d%s" % (i, desc) + nl)
        if wrap and L:
            w = int(rng.integers(10, 80))
            for j in range(0, L, w):
                piece = seq[j:j + w]
                if i % 7 == 3:
                    piece = piece[:3] + b" " + piece[3:]  # spaces inside lines are dropped
                out.append(piece + (b"  " if i % 5 == 1 else b"") + nl)
        elif L:
            out.append(seq + nl)
    return b"".join(out)


def _fastq_text(rng, n, crlf=False, blank=False) -> bytes:
    nl = b"\r\n" if crlf else b"\n"
    out = []
    for i in range(n):
        L = int(rng.integers(0, 300))
        seq = _pick(rng, b"ACGTN", L)
        qual = _pick(rng, b"@+!#ABCDEFGHIJ", L)  # '@' / '+' start quality lines too
        cap = b"read_%d x" % i if i % 3 == 0 else b""
        out.append(b"@read_%d x" % i + nl + seq + nl + b"+" + cap + nl + qual + nl)
        if blank and i % 11 == 0:
            out.append(nl)
    return b"".join(out)


def _wrapped_fastq(rng, n) -> bytes:
    out = []
    for i in range(n):
        L = int(rng.integers(1, 200))
        seq = _pick(rng, b"ACGT", L)
        qual = _pick(rng, b"@+IJ", L)
        w = 60
        out.append(b"@w%d\n" % i + b"\n".join(seq[j:j + w] for j in range(0, L, w)) + b"\n+\n"
                   + b"\n".join(qual[j:j + w] for j in range(0, L, w)) + b"\n")
    return b"".join(out)


def _native(path, max_bytes, threads=0):
    got = []
    with FastxReader(path, threads=threads) as rd:
        for b in rd.batches(max_bytes):
            buf, o = b.packed.buf, b.packed.offsets.tolist()
            raw = buf[:o[-1]].tobytes()
            got += [(i.encode(), raw[o[j]:o[j + 1]]) for j, i in enumerate(b.ids())]
    return got


@pytest.mark.parametrize("crlf", [False, True])
@pytest.mark.parametrize("max_bytes", [1, 4096, 1 << 30])
def test_fasta_matches_restatement(tmp_path, crlf, max_bytes):
    rng = np.random.default_rng(7 + crlf)
    p = tmp_path / "x.fasta"
    p.write_bytes(_fasta_text(rng, 3000, crlf=crlf))
    want = ofx.parse_file(p)
    assert _native(p, max_bytes) == want


@pytest.mark.parametrize("max_bytes", [1, 5000, 1 << 30])
def test_fastq_matches_restatement(tmp_path, max_bytes):
    rng = np.random.default_rng(3)
    p = tmp_path / "x.fq"
    p.write_bytes(_fastq_text(rng, 4000, blank=True))
    want = ofx.parse_file(p)
    assert _native(p, max_bytes) == want


def test_multithreaded_split_large_files(tmp_path):
    """> 1 MiB per part: batches are cut into many parts parsed concurrently."""
    rng = np.random.default_rng(11)
    fa = tmp_path / "big.fa"
    fa.write_bytes(_fasta_text(rng, 60_000, junk=False))
    fq = tmp_path / "big.fastq"
    fq.write_bytes(_fastq_text(rng, 60_000, crlf=True))
    assert fa.stat().st_size > 8 << 20 and fq.stat().st_size > 8 << 20
    for p in (fa, fq):
        want = ofx.parse_file(p)
        for threads in (1, 8):
            for mb in (3 << 20, 1 << 30):
                assert _native(p, mb, threads) == want


def test_wrapped_fastq_is_parsed_sequentially(tmp_path):
    p = tmp_path / "w.fastq"
    p.write_bytes(_wrapped_fastq(np.random.default_rng(5), 20_000))
    want = ofx.parse_file(p)
    assert _native(p, 1 << 30, 8) == want
    assert _native(p, 10_000, 8) == want


@pytest.mark.parametrize("text,msg", [
    (b"ACGT\n", "should start with '@'"),
    (b"@a\nACGT\n", "End of file without quality"),
    (b"@a\n", "Unexpected end of file"),
    (b"@a\nACGT\n+b\nIIII\n", "captions differ"),
    (b"@a\nAC GT\n+\nIIIII\n", "Whitespace is not allowed"),
    (b"@a\nACGT\n+\nIII\n", "Lengths of sequence and quality"),
])
def test_fastq_errors_match(tmp_path, text, msg):
    p = tmp_path / "bad.fq"
    p.write_bytes(text)
    with pytest.raises(ValueError, match=msg):
        ofx.parse_file(p)
    with pytest.raises(ValueError, match=msg):
        _native(p, 1 << 30)


def test_empty_and_headerless_files(tmp_path):
    for name, text in [("e.fasta", b""), ("n.fasta", b"no records here\n"), ("e.fq", b""), ("b.fq", b"\n\n")]:
        p = tmp_path / name
        p.write_bytes(text)
        assert _native(p, 1 << 20) == ofx.parse_file(p) == []


def _rows(b):
    o = b.packed.offsets.tolist()
    raw = b.packed.buf[:o[-1]].tobytes()
    return [(i.encode(), raw[o[j]:o[j + 1]]) for j, i in enumerate(b.ids())]


def test_double_buffered_batches_stay_valid(tmp_path):
    """A batch stays intact while the next one is parsed (xs_fastx_next contract)."""
    rng = np.random.default_rng(2)
    p = tmp_path / "d.fasta"
    p.write_bytes(_fasta_text(rng, 2000, junk=False))
    want = ofx.parse_file(p)
    seen = []
    with FastxReader(p) as rd:
        prev = rd.next_batch(20_000)
        while prev.n:
            cur = rd.next_batch(20_000)  # parsed into the other buffer
            seen += _rows(prev)
            prev = cur
    assert seen == want
    # the pipelined generator yields the same records
    assert [r for b in read_batches(p, max_bytes=20_000) for r in _rows(b)] == want


def test_get_record_iterator_contract(tmp_path):
    with pytest.raises(ValueError, match="Path object"):
        get_record_iterator(str(tmp_path))
    with pytest.raises(ValueError, match="does not exist"):
        get_record_iterator(tmp_path / "missing.fasta")
    with pytest.raises(ValueError, match="must be a file"):
        get_record_iterator(tmp_path)
    bad = tmp_path / "x.txt"
    bad.write_text(">a\nAC\n")
    with pytest.raises(ValueError, match="Invalid file format"):
        get_record_iterator(bad)
    ok = tmp_path / "x.fna"
    ok.write_text(">a b\nAC\nGT\n>c\nT\n")
    assert [(r.id, r.seq) for r in get_record_iterator(ok)] == [("a", "ACGT"), ("c", "T")]


def _native_part(path, part, parts, max_bytes=1 << 30, threads=0):
    got = []
    with FastxReader(path, threads=threads, part=part, parts=parts) as rd:
        for b in rd.batches(max_bytes):
            got += _rows(b)
    return got


@pytest.mark.parametrize("kind", ["fasta", "fasta_crlf", "fastq", "fastq_blank", "fastq_wrapped", "tiny"])
def test_byte_range_parts_stitch_to_the_whole_file(tmp_path, kind):
    """xs_fastx_open_range: each rank of a read-sharded job parses only its
    part of the file; the parts, concatenated in part order, are exactly the
    whole file's records (ids and sequences), for 1-9 parts, more parts than
    records, every batch size and thread count."""
    rng = np.random.default_rng(len(kind))
    text = {"fasta": lambda: _fasta_text(rng, 3000),
            "fasta_crlf": lambda: _fasta_text(rng, 2000, crlf=True),
            "fastq": lambda: _fastq_text(rng, 3000),
            "fastq_blank": lambda: _fastq_text(rng, 3000, crlf=True, blank=True),
            "fastq_wrapped": lambda: _wrapped_fastq(rng, 3000),
            "tiny": lambda: b">a\nACGT\n>b\nGG\n"}[kind]()
    p = tmp_path / ("x.fq" if "fastq" in kind else "x.fasta")
    p.write_bytes(text)
    want = ofx.parse_file(p)
    for parts in (1, 2, 3, 5, 9):
        got = [_native_part(p, i, parts, mb, th) for i in range(parts)
               for mb, th in [((1 << 30) if i % 2 else 7000, 1 + i % 3)]]
        assert [r for g in got for r in g] == want, parts
        if len(want) >= 100 and parts > 1:
            sizes = [len(g) for g in got]
            assert min(sizes) > 0 and max(sizes) <= 2 * len(want) / parts + 10  # balanced by bytes
    with pytest.raises(ValueError):
        FastxReader(p, part=3, parts=3)


def test_byte_range_parts_of_a_large_file(tmp_path):
    """Parts larger than 1 MiB are themselves parsed by several threads."""
    rng = np.random.default_rng(17)
    p = tmp_path / "big.fastq"
    p.write_bytes(_fastq_text(rng, 60_000))
    want = ofx.parse_file(p)
    got = [r for i in range(3) for r in _native_part(p, i, 3, 3 << 20, 8)]
    assert got == want
