"""Pure-Python restatement of Biopython's FASTA / FASTQ record parsing.

TEST INFRASTRUCTURE ONLY: the checker for the native reader
(xspect2_amd/csrc/xs_fastx.cpp, xs_fastx_* in include/xspect_hip.h).  Only
tests/ may import it.

The reference parses input files with ``Bio.SeqIO.parse(path, "fasta"|"fastq")``
(src/xspect/file_io.py:47-79).  Biopython is not installed offline, so this
restates its SimpleFastaParser / FastqGeneralIterator behaviour as used there
(parity unpinned against Biopython itself):

* FASTA: text before the first ``>`` line is skipped; title = header line
  without ``>`` and right-stripped; id = ``title.split(None, 1)[0]`` (or "");
  sequence = the record's lines, each right-stripped, joined, with " " and
  "\\r" removed.
* FASTQ: blank lines between records are skipped; a header must start with
  ``@``; sequence lines run to the first line starting with ``+`` (a non-empty
  caption there must equal the title); the sequence may not contain " " or
  "\\t"; quality lines are read until they hold >= len(sequence) characters and
  must hold exactly that many.

Lines are split at "\\n" only (files are read as bytes).
"""
from __future__ import annotations

from pathlib import Path

_WS = b" \t\n\r\x0b\x0c\x1c\x1d\x1e\x1f"


def _rstrip(line: bytes) -> bytes:
    return line.rstrip(_WS)


def _first_token(title: bytes) -> bytes:
    parts = title.split(None, 1)
    return parts[0] if parts else b""


def parse_fasta(data: bytes) -> list[tuple[bytes, bytes]]:
    """[(id, sequence)] of a FASTA text."""
    out = []
    title = None
    chunks: list[bytes] = []
    for line in data.split(b"\n"):
        if line.startswith(b">"):
            if title is not None:
                out.append((_first_token(title), b"".join(chunks).replace(b" ", b"").replace(b"\r", b"")))
            title = _rstrip(line[1:])
            chunks = []
        elif title is not None:
            chunks.append(_rstrip(line))
    if title is not None:
        out.append((_first_token(title), b"".join(chunks).replace(b" ", b"").replace(b"\r", b"")))
    return out


def parse_fastq(data: bytes) -> list[tuple[bytes, bytes]]:
    """[(id, sequence)] of a FASTQ text; raises ValueError like Biopython."""
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()  # the text's final newline
    out = []
    i, n = 0, len(lines)
    while i < n:
        if _rstrip(lines[i]) == b"":
            i += 1
            continue
        head = lines[i]
        i += 1
        if not head.startswith(b"@"):
            raise ValueError("Records in Fastq files should start with '@' character")
        title = _rstrip(head[1:])
        seq = []
        while i < n and not lines[i].startswith(b"+"):
            seq.append(_rstrip(lines[i]))
            i += 1
        s = b"".join(seq)
        if i >= n:
            raise ValueError("End of file without quality information." if s else "Unexpected end of file")
        caption = _rstrip(lines[i][1:])
        i += 1
        if caption and caption != title:
            raise ValueError("Sequence and quality captions differ.")
        if b" " in s or b"\t" in s:
            raise ValueError("Whitespace is not allowed in the sequence.")
        q = 0
        while q < len(s) and i < n:
            q += len(_rstrip(lines[i]))
            i += 1
        if q != len(s):
            raise ValueError("Lengths of sequence and quality values differs")
        out.append((_first_token(title), s))
    return out


def parse_file(path: Path) -> list[tuple[bytes, bytes]]:
    data = Path(path).read_bytes()
    return parse_fastq(data) if Path(path).suffix[1:] in ("fastq", "fq") else parse_fasta(data)


def parse_titles(path: Path) -> list[bytes]:
    """Record titles (header line minus '>' / '@', right-stripped), in file
    order: SeqRecord.description as Bio.SeqIO.parse sets it."""
    data = Path(path).read_bytes()
    fastq = Path(path).suffix[1:] in ("fastq", "fq")
    out = []
    if not fastq:
        for line in data.split(b"\n"):
            if line.startswith(b">"):
                out.append(_rstrip(line[1:]))
        return out
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    i, n = 0, len(lines)
    while i < n:  # well-formed input: the same walk as parse_fastq
        if _rstrip(lines[i]) == b"":
            i += 1
            continue
        out.append(_rstrip(lines[i][1:]))
        i += 1
        s = 0
        while i < n and not lines[i].startswith(b"+"):
            s += len(_rstrip(lines[i]))
            i += 1
        i += 1
        q = 0
        while q < s and i < n:
            q += len(_rstrip(lines[i]))
            i += 1
    return out


def write_fasta_bio(records, path: Path, width: int = 60, append: bool = False) -> None:
    """Bio.SeqIO.write(record, handle, "fasta") restated (FastaWriter): the
    title is the description when its first token is the id, else
    "id description", else the id; then the sequence in lines of `width`
    characters (none for an empty sequence).  records: (id, description, seq)
    bytes triples."""
    with open(path, "ab" if append else "wb") as fh:
        for rid, desc, seq in records:
            rid = rid.replace(b"\n", b" ").replace(b"\r", b" ")
            desc = desc.replace(b"\n", b" ").replace(b"\r", b" ")
            if desc and desc.split(None, 1)[0] == rid:
                title = desc
            elif desc:
                title = rid + b" " + desc
            else:
                title = rid
            fh.write(b">" + title + b"\n")
            for i in range(0, len(seq), width):
                fh.write(seq[i:i + width] + b"\n")
