"""Device mode of the native reader (xs_fastx_open_device / _next_device,
xs_fastx_dev.hip) against its host mode and the pure-Python restatement of
Biopython's parsers (oracle/fastx.py) (GPU).

Every batch of the device mode must equal the host mode's batch for the same
window: record count, sequence bytes and offsets, ids, titles, file offsets.
Windows the device rules do not cover (blank lines between FASTQ records,
wrapped FASTQ, ' ' or '\\r' inside FASTA lines, malformed records) go through
the host parser, which the flag ``parsed_on_device`` shows; error messages
are the host reader's.  Then the probe on a device batch
(xs_query_hits_device) equals the probe on the host batch.
"""
from __future__ import annotations

import numpy as np
import pytest

import fastx as ofx  # test-only checker (oracle/fastx.py)
from test_fastx import _fasta_text, _fastq_text, _pick, _wrapped_fastq

from xspect2_amd.file_io import FastxReader, read_batches

pytestmark = pytest.mark.gpu


def _batches(path, max_bytes, device, part=0, parts=1, threads=0):
    out = []
    with FastxReader(path, threads=threads, part=part, parts=parts, device=device) as rd:
        for b in rd.batches(max_bytes):
            pr = b.to_host() if device is not None else b.packed
            o = pr.offsets.astype(np.int64)
            raw = pr.buf[:o[-1]].tobytes() if b.n else b""
            out.append({"n": b.n, "offsets": o.tolist(), "seqs": raw, "ids": b.ids(),
                        "descs": b.descriptions(), "text_offset": b.text_offset,
                        "dev": getattr(b, "parsed_on_device", None)})
    return out


def _same(path, max_bytes, part=0, parts=1, threads=0):
    host = _batches(path, max_bytes, None, part, parts, threads)
    dev = _batches(path, max_bytes, 0, part, parts, threads)
    assert len(dev) == len(host)
    for h, d in zip(host, dev):
        for key in ("n", "offsets", "seqs", "ids", "descs", "text_offset"):
            assert d[key] == h[key], key
    return dev


def _records(batches):
    return [(i.encode(), b["seqs"][b["offsets"][j]:b["offsets"][j + 1]])
            for b in batches for j, i in enumerate(b["ids"])]


def _plain_fastq(rng, n, crlf=False, caption=True, tail_newline=True) -> bytes:
    nl = b"\r\n" if crlf else b"\n"
    out = []
    for i in range(n):
        L = int(rng.integers(1, 300))
        seq = _pick(rng, b"ACGTNacgt", L)
        qual = _pick(rng, b"@+!#ABCDEFGHIJ", L)
        title = [b"r%d" % i, b"r%d some desc" % i, b"  r%d\tx " % i, b"r%d\x1f" % i][i % 4]
        cap = title.rstrip() if caption and i % 3 == 0 else b""
        out.append(b"@" + title + nl + seq + nl + b"+" + cap + nl + qual + nl)
    text = b"".join(out)
    return text if tail_newline else text.rstrip(b"\r\n")


@pytest.mark.parametrize("crlf", [False, True])
@pytest.mark.parametrize("max_bytes", [1, 5000, 1 << 30])
def test_fastq_device_equals_host(tmp_path, crlf, max_bytes):
    rng = np.random.default_rng(31 + crlf)
    p = tmp_path / "x.fq"
    p.write_bytes(_plain_fastq(rng, 3000, crlf=crlf))
    dev = _same(p, max_bytes)
    assert all(b["dev"] for b in dev), "plain 4-line FASTQ is parsed on the device"
    assert _records(dev) == ofx.parse_file(p)


def test_fastq_last_line_without_newline(tmp_path):
    p = tmp_path / "t.fastq"
    p.write_bytes(_plain_fastq(np.random.default_rng(2), 500, tail_newline=False))
    dev = _same(p, 1 << 30)
    assert dev[0]["dev"] and _records(dev) == ofx.parse_file(p)


@pytest.mark.parametrize("max_bytes", [1, 5000, 1 << 30])
def test_fasta_device_equals_host(tmp_path, max_bytes):
    """Wrapped lines, CRLF, lower case, empty records, titles with tabs,
    leading text; the generator's ' ' inside some lines sends those windows
    to the host parser."""
    for crlf in (False, True):
        rng = np.random.default_rng(7 + crlf)
        p = tmp_path / f"x{int(crlf)}.fasta"
        p.write_bytes(_fasta_text(rng, 3000, crlf=crlf))
        dev = _same(p, max_bytes)
        assert _records(dev) == ofx.parse_file(p)


def test_fasta_without_spaces_is_parsed_on_device(tmp_path):
    rng = np.random.default_rng(12)
    out = [b"junk before the first record\n"]
    for i in range(2000):
        L = int(rng.integers(0, 900))
        seq = _pick(rng, b"ACGTNacgtn", L)
        out.append(b">c%d len=%d\n" % (i, L) + b"".join(seq[j:j + 70] + b"\n" for j in range(0, L, 70)))
    p = tmp_path / "g.fna"
    p.write_bytes(b"".join(out)[:-1])  # no final newline
    for mb in (4096, 1 << 30):
        dev = _same(p, mb)
        assert all(b["dev"] for b in dev)
        assert _records(dev) == ofx.parse_file(p)


def test_fallback_windows_and_wrapped_fastq(tmp_path):
    rng = np.random.default_rng(3)
    blank = tmp_path / "blank.fq"  # blank lines between records: host parser
    blank.write_bytes(_fastq_text(rng, 3000, blank=True))
    dev = _same(blank, 1 << 30)
    assert not dev[0]["dev"] and _records(dev) == ofx.parse_file(blank)
    wrapped = tmp_path / "w.fastq"
    wrapped.write_bytes(_wrapped_fastq(rng, 3000))
    for mb in (10_000, 1 << 30):
        dev = _same(wrapped, mb)
        assert not any(b["dev"] for b in dev) and _records(dev) == ofx.parse_file(wrapped)
    empty_seq = tmp_path / "e.fq"  # an empty sequence: host parser
    empty_seq.write_bytes(b"@a\nACGT\n+\nIIII\n@b\n\n+\n\n@c\nAC\n+\nII\n")
    dev = _same(empty_seq, 1 << 30)
    assert _records(dev) == ofx.parse_file(empty_seq)


@pytest.mark.parametrize("text,msg", [
    (b"ACGT\n", "should start with '@'"),
    (b"@a\nACGT\n", "End of file without quality"),
    (b"@a\n", "Unexpected end of file"),
    (b"@a\nACGT\n+b\nIIII\n", "captions differ"),
    (b"@a\nAC GT\n+\nIIIII\n", "Whitespace is not allowed"),
    (b"@a\nACGT\n+\nIII\n", "Lengths of sequence and quality"),
    (b"@a\nACGT\n+\nIIII\n@b\nAC\tG\n+\nIIII\n", "Whitespace is not allowed"),
])
def test_fastq_errors_match_host(tmp_path, text, msg):
    p = tmp_path / "bad.fq"
    p.write_bytes(text)
    with pytest.raises(ValueError, match=msg):
        _batches(p, 1 << 30, None)
    with pytest.raises(ValueError, match=msg):
        _batches(p, 1 << 30, 0)


def test_empty_and_headerless(tmp_path):
    for name, text in [("e.fasta", b""), ("n.fasta", b"no records here\n"), ("e.fq", b""), ("b.fq", b"\n\n")]:
        p = tmp_path / name
        p.write_bytes(text)
        assert _batches(p, 1 << 20, 0) == []


@pytest.mark.parametrize("kind", ["fq", "fasta"])
def test_byte_range_parts(tmp_path, kind):
    rng = np.random.default_rng(9)
    p = tmp_path / f"x.{kind}"
    p.write_bytes(_plain_fastq(rng, 5000) if kind == "fq" else _fasta_text(rng, 5000, junk=False))
    want = ofx.parse_file(p)
    got = []
    for part in range(3):
        got += _records(_same(p, 20_000, part, 3))
    assert got == want


def test_large_windows_many_tiles(tmp_path):
    """~40 MB of FASTQ: windows span thousands of 16 KiB tiles and several
    4 MiB pieces of the pinned text load; reads of 150 bp as in config 2."""
    rng = np.random.default_rng(42)
    n = 120_000
    seqs = rng.integers(0, 4, (n, 150), dtype=np.uint8)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    lines = [b"@read_%d\n%s\n+\n%s\n" % (i, acgt[seqs[i]].tobytes(), b"I" * 150) for i in range(n)]
    p = tmp_path / "r.fastq"
    p.write_bytes(b"".join(lines))
    for mb in (7 << 20, 1 << 30):
        dev = _same(p, mb, threads=8)
        assert all(b["dev"] for b in dev)
        assert sum(b["n"] for b in dev) == n


def test_batch_size_changes_between_calls(tmp_path):
    """The reader loads up to two windows ahead for the batch size of the
    last call; a caller that changes the size gets the windows of the new
    size (the queued loads are finished and dropped), as the host reader."""
    rng = np.random.default_rng(21)
    p = tmp_path / "r.fastq"
    p.write_bytes(_plain_fastq(rng, 4000))
    sizes = [9000, 9000, 3000, 50_000, 50_000, 700, 1 << 20]

    def run(device):
        got = []
        with FastxReader(p, device=device) as rd:
            for k in range(64):
                b = rd.next_batch(sizes[k % len(sizes)])
                if b.n == 0:
                    break
                pr = b.to_host() if device is not None else b.packed
                o = pr.offsets.astype(np.int64)
                got.append((b.n, b.text_offset, pr.buf[:o[-1]].tobytes(), b.ids()))
        return got

    host, dev = run(None), run(0)
    assert len(dev) == len(host) > 5
    assert dev == host


@pytest.mark.parametrize("inject", [None, b" ", b"\r"])
def test_fasta_unwrapped_megabase_lines(tmp_path, inject):
    """Assemblies written one sequence line per contig: 2-3 Mbp lines are
    checked by whole waves; a ' ' or '\\r' inside one sends the window to the
    host parser, which removes it, as Biopython does."""
    rng = np.random.default_rng(11)
    contigs = [_pick(rng, b"ACGT", L) for L in (3_000_000, 17, 2_000_003, 150)]
    if inject is not None:
        c = bytearray(contigs[2])
        c[1_234_567] = inject[0]
        contigs[2] = bytes(c)
    p = tmp_path / "asm.fasta"
    p.write_bytes(b"".join(b">ctg%d len=%d\n%s\n" % (i, len(c), c) for i, c in enumerate(contigs)))
    dev = _same(p, 1 << 30)
    assert all(b["dev"] for b in dev) == (inject is None)
    assert sum(b["n"] for b in dev) == 4


def test_kept_device_sides_across_opens(tmp_path):
    """Closed readers hand their device side (streams, buffers at their grown
    sizes) to the next open: a large file, then small ones, then two readers
    open at once and read in turns, each batch equal to the host reader's."""
    rng = np.random.default_rng(9)
    big = tmp_path / "big.fastq"
    n = 60_000
    seqs = rng.integers(0, 4, (n, 150), dtype=np.uint8)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    big.write_bytes(b"".join(b"@b%d\n%s\n+\n%s\n" % (i, acgt[seqs[i]].tobytes(), b"I" * 150) for i in range(n)))
    small_fq = tmp_path / "s.fastq"
    small_fq.write_bytes(_plain_fastq(rng, 500))
    small_fa = tmp_path / "s.fasta"
    small_fa.write_bytes(b"".join(b">c%d x\n%s\n" % (i, _pick(rng, b"ACGT", 200)) for i in range(300)))
    for path, mb in ((big, 1 << 30), (small_fq, 1 << 30), (small_fa, 3000), (big, 4 << 20), (small_fq, 700)):
        _same(path, mb)
    want = {p: _batches(p, 5000, None) for p in (small_fq, small_fa)}
    ra, rb = FastxReader(small_fq, device=0), FastxReader(small_fa, device=0)
    try:
        got = {small_fq: [], small_fa: []}
        live = [(ra, small_fq), (rb, small_fa)]
        while live:
            for rd, p in list(live):
                b = rd.next_batch(5000)
                if b.n == 0:
                    live.remove((rd, p))
                    continue
                pr = b.to_host()
                o = pr.offsets.astype(np.int64)
                got[p].append((b.n, o.tolist(), pr.buf[:o[-1]].tobytes(), b.ids(), b.descriptions()))
        for p in got:
            assert got[p] == [(h["n"], h["offsets"], h["seqs"], h["ids"], h["descs"]) for h in want[p] if h["n"]]
    finally:
        ra.close()
        rb.close()


def test_probe_on_device_batches_equals_host(tmp_path, oracle_mod):
    from xspect2_amd.bank import Bank
    from xspect2_amd.synth import make_genomes, make_reads
    D, k = 12, 21
    genomes = make_genomes(D, 30_000, seed=4)
    sig = [oracle_mod.signature_size(30_000, 7, 0.01)]
    gb = Bank.create_cobs(k, 7, sig, D, [f"s{i}" for i in range(D)])
    gb.build([g.tobytes() for g in genomes], list(range(D)))
    reads, _ = make_reads(genomes, 20_000, 150, seed=6)
    p = tmp_path / "r.fq"
    p.write_bytes(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, reads[i].tobytes(), b"I" * 150) for i in range(len(reads))))
    from xspect2_amd.packing import PackedReads
    host = [PackedReads(b.packed.buf.copy(), b.packed.offsets.copy())  # a batch's buffers are reused
            for b in read_batches(p, 1 << 20)]
    for step in (1, 3):
        hb = iter(host)
        for b in read_batches(p, 1 << 20, device=0):
            pr = next(hb)
            h_dev, n_dev = gb.query(b, step=step, hit_dtype="auto")
            h_host, n_host = gb.query(pr, step=step, hit_dtype="auto")
            assert h_dev.dtype == h_host.dtype == np.uint8
            assert np.array_equal(h_dev, h_host) and np.array_equal(n_dev, n_host)
            t_dev, k_dev = gb.query_totals(b, step=step)
            t_host, k_host = gb.query_totals(pr, step=step)
            assert np.array_equal(t_dev, t_host) and k_dev == k_host
    gb.close()


def test_stale_device_batches_are_refused(tmp_path):
    """A device batch outlives neither its reader nor the reader's second
    following batch: using it then raises instead of reading freed HBM."""
    from xspect2_amd.bank import Bank
    p = tmp_path / "r.fq"
    p.write_bytes(_plain_fastq(np.random.default_rng(5), 3000))
    gb = Bank.create_cobs(21, 7, [5000], 8, [f"s{i}" for i in range(8)])
    with FastxReader(p, device=0) as rd:
        b0 = rd.next_batch(20_000)
        b1 = rd.next_batch(20_000)
        gb.query(b0)  # still valid: one batch since
        rd.next_batch(20_000)
        with pytest.raises(RuntimeError, match="no longer valid"):
            gb.query(b0)
        gb.query_totals(b1)
    with pytest.raises(RuntimeError, match="no longer valid"):
        gb.query_totals(b1)
    with pytest.raises(RuntimeError, match="no longer valid"):
        b1.to_host()
    gb.close()


def _outcome(path, max_bytes, device):
    """The batches of a reader mode, or ('error', message) where it raises."""
    try:
        return _batches(path, max_bytes, device)
    except ValueError as e:
        return ("error", str(e))


def _mutate(rng, text: bytes) -> bytes:
    """One of: truncation at a random byte, random bytes spliced in (record
    markers, whitespace, CR, bases), a blank line inserted, a line dropped."""
    if not text:
        return text
    kind = int(rng.integers(0, 4))
    pos = int(rng.integers(0, len(text)))
    if kind == 0:
        return text[:pos]
    if kind == 1:
        junk = _pick(rng, b"\n@+> \r\tACGTN", int(rng.integers(1, 6)))
        return text[:pos] + junk + text[pos:]
    nl = text.find(b"\n", pos)
    if nl < 0:
        return text
    if kind == 2:
        return text[:nl + 1] + b"\n" + text[nl + 1:]
    nxt = text.find(b"\n", nl + 1)
    return text[:nl + 1] + (text[nxt + 1:] if nxt >= 0 else b"")


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_device_equals_host(tmp_path, seed):
    """Malformed and well-formed inputs (the host sanitizer sweep's kinds:
    truncations, spliced bytes, blank lines, dropped lines) in both formats
    and at several window sizes: the device mode gives the host mode's batches,
    or raises the host mode's error."""
    rng = np.random.default_rng(1000 + seed)
    kind = ["fq", "fasta", "fq_plain"][seed % 3]
    n = int(rng.integers(1, 400))
    if kind == "fasta":
        text, ext = _fasta_text(rng, n, wrap=bool(seed % 2), crlf=seed % 4 == 1), "fasta"
    elif kind == "fq":
        text, ext = _fastq_text(rng, n, crlf=seed % 4 == 0, blank=seed % 5 == 0), "fq"
    else:
        text, ext = _plain_fastq(rng, n, crlf=seed % 2 == 1, tail_newline=seed % 3 != 0), "fastq"
    for _ in range(int(rng.integers(0, 4))):
        text = _mutate(rng, text)
    p = tmp_path / f"f.{ext}"
    p.write_bytes(text)
    for mb in (int(rng.integers(1, 3000)), 50_000, 1 << 30):
        host = _outcome(p, mb, None)
        dev = _outcome(p, mb, 0)
        if isinstance(host, tuple):
            assert dev == host, (mb, host, dev if isinstance(dev, tuple) else "batches")
            continue
        assert not isinstance(dev, tuple), (mb, dev)
        assert len(dev) == len(host)
        for h, d in zip(host, dev):
            for key in ("n", "offsets", "seqs", "ids", "descs", "text_offset"):
                assert d[key] == h[key], (mb, key)
