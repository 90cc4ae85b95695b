"""FASTA/FASTQ records without Biopython (host side of the probe path).

Mirrors what the hot path consumes from ``src/xspect/file_io.py:47-79``
(``get_record_iterator``: Bio.SeqIO parse by file extension).  A record has
``.id`` (first whitespace token of the header, as Bio.SeqIO) and ``.seq``.
Bio.SeqRecord objects are accepted anywhere a record is expected.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Iterator

FASTA_ENDINGS = ["fasta", "fna", "fa", "ffn", "frn"]  # definitions.py:6
FASTQ_ENDINGS = ["fastq", "fq"]                       # definitions.py:7


@dataclass
class Record:
    id: str
    seq: str
    description: str = ""

    def __len__(self) -> int:
        return len(self.seq)


def is_record(obj) -> bool:
    return hasattr(obj, "id") and hasattr(obj, "seq")


def seq_text(obj) -> str:
    """The sequence text of a str / bytes / Bio.Seq."""
    if isinstance(obj, str):
        return obj
    if isinstance(obj, (bytes, bytearray)):
        return bytes(obj).decode("ascii")
    return str(obj)


def _fasta(path: Path) -> Iterator[Record]:
    rid, desc, chunks = None, "", []
    with open(path, "r", encoding="utf-8") as fh:
        for line in fh:
            if line.startswith(">"):
                if rid is not None:
                    yield Record(rid, "".join(chunks), desc)
                desc = line[1:].rstrip("\r\n")
                rid = desc.split(None, 1)[0] if desc.strip() else ""
                chunks = []
            elif rid is not None:
                chunks.append(line.strip())
    if rid is not None:
        yield Record(rid, "".join(chunks), desc)


def _fastq(path: Path) -> Iterator[Record]:
    with open(path, "r", encoding="utf-8") as fh:
        while True:
            head = fh.readline()
            if not head:
                return
            if not head.strip():
                continue
            if not head.startswith("@"):
                raise ValueError(f"{path}: records in FASTQ files should start with '@'")
            desc = head[1:].rstrip("\r\n")
            seq_lines = []
            line = fh.readline()
            while line and not line.startswith("+"):
                seq_lines.append(line.strip())
                line = fh.readline()
            seq = "".join(seq_lines)
            qual = []
            got = 0
            while got < len(seq):
                q = fh.readline()
                if not q:
                    raise ValueError(f"{path}: truncated FASTQ record {desc!r}")
                q = q.strip()
                qual.append(q)
                got += len(q)
            yield Record(desc.split(None, 1)[0] if desc.strip() else "", seq, desc)


def get_record_iterator(file_path: Path) -> Iterator[Record]:
    """Record iterator of a FASTA/FASTQ file (error messages as file_io.py:66-79)."""
    if not isinstance(file_path, Path):
        raise ValueError("Path must be a Path object")
    if not file_path.exists():
        raise ValueError("File does not exist")
    if not file_path.is_file():
        raise ValueError("Path must be a file")
    ending = file_path.suffix[1:]
    if ending in FASTA_ENDINGS:
        return _fasta(file_path)
    if ending in FASTQ_ENDINGS:
        return _fastq(file_path)
    raise ValueError("Invalid file format, must be a fasta or fastq file")


def write_fasta(records, path: Path, width: int = 0) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", encoding="utf-8") as fh:
        for r in records:
            s = seq_text(r.seq)
            fh.write(f">{r.id}\n")
            if width:
                for i in range(0, len(s), width):
                    fh.write(s[i:i + width] + "\n")
            else:
                fh.write(s + "\n")


def prepare_input_output_paths(input_path: Path):
    """Input files + output-path factory (mirror of file_io.py:194-234).

    A directory yields its files grouped by ending in the order of
    FASTA_ENDINGS + FASTQ_ENDINGS (sorted within an ending, where the reference
    keeps glob order) and suffixes every output name with _<idx+1>.
    """
    input_path = Path(input_path)
    input_is_dir = input_path.is_dir()
    if input_is_dir:
        inputs = [p for e in FASTA_ENDINGS + FASTQ_ENDINGS for p in sorted(input_path.glob(f"*.{e}"))]
    elif input_path.is_file():
        inputs = [input_path]
    else:
        raise ValueError("Invalid input path")

    def get_output_path(idx: int, output_path: Path) -> Path:
        output_path = Path(output_path)
        if input_is_dir:
            return output_path.parent / f"{output_path.stem}_{idx + 1}{output_path.suffix}"
        return output_path

    return inputs, get_output_path
