"""MLST scheme model: one COBS compact bank per locus, resident in HBM.

Drop-in for ``xspect.models.probabilistic_filter_mlst_model.ProbabilisticFilterMlstSchemeModel``
(reference ``src/xspect/models/probabilistic_filter_mlst_model.py:22-449``).
Semantics kept: sequences shorter than 10 kbp are one query per locus whose
first result is the top allele (``:272-286``); longer ones are split by
``sequence_splitter`` (``:382-426``), each chunk keeps alleles scoring > 50
(``get_cobs_result`` ``:362-380``), kept scores are summed per allele and
stably sorted by -score (``:248-256``).  What changes: every chunk of every
record of a locus (and every short record) is probed in one batched GPU call
(xs_mlst_query) instead of one COBS call per chunk, and the > 50 chunk sums
are made on the device.  The PubMLST strain-type POST (``:295-302``) is network I/O and is
delegated to ``strain_type_resolver``.
"""
from __future__ import annotations

import json
from collections import namedtuple
from pathlib import Path

import numpy as np

from ._lib import XS_BANK_COBS_COMPACT
from .bank import Bank, cobs_signature_size
from .file_io import get_record_iterator, is_record, seq_text
from .packing import pack_sequences
from .probabilistic_filter_model import ProbabilisticFilterModel
from .result import MlstResult
from .util import slugify

SearchResult = namedtuple("SearchResult", ["doc_name", "score"])

LONG_SEQUENCE = 10_000        # :236
CHUNK_KMER_THRESHOLD = 50     # :378
DEFAULT_PAGE_SIZE = 64        # bytes per row per doc group = one 64-B line


def _default_resolver(flattened: dict, scheme_url: str):
    """ST name lookup through XspecT's PubMLST handler when it is importable."""
    try:
        from xspect.handlers.pubmlst import PubMLSTHandler  # type: ignore
    except Exception:
        return None
    return PubMLSTHandler().get_strain_type_name(flattened, scheme_url)


def first_allele_length(locus_path: Path) -> int:
    """Length of the first record of the first ``*.fasta`` file that
    ``locus_path.glob`` yields (directory order, not sorted), which the
    reference stores as the locus' "average" size (:126-130).  It sets the
    splitter's chunk width and ``has_sufficient_score``'s threshold."""
    fasta_file_path = next(locus_path.glob("*.fasta"), None)
    if fasta_file_path is None:
        raise ValueError(f"No allele FASTA files in {locus_path}")
    return len(next(get_record_iterator(fasta_file_path)).seq)


class ProbabilisticFilterMlstSchemeModel(ProbabilisticFilterModel):
    """One compact bank per locus of an MLST scheme."""

    def __init__(self, k: int, model_display_name: str, base_path: Path, scheme_url: str,
                 organism: str, fpr: float = 0.001, num_hashes: int = 1,
                 author: str | None = None, author_email: str | None = None,
                 model_type: str = "MLST") -> None:
        super().__init__(k, model_display_name, author, author_email, model_type, base_path, fpr,
                         num_hashes, None)
        self.organism = organism
        self.scheme_url = scheme_url
        self.loci: dict[str, int] = {}
        self.avg_locus_bp_size: list[int] = []
        self.indices: list[Bank] = []
        self.strain_type_resolver = _default_resolver

    def to_dict(self) -> dict:
        return super().to_dict() | {"organism": self.organism, "scheme_url": self.scheme_url,
                                    "loci": self.loci,
                                    "average_locus_base_pair_size": self.avg_locus_bp_size}

    def slug(self) -> str:
        return slugify(self.organism + "-" + self.model_display_name + "-" + self.model_type)

    def get_cobs_index_path(self, locus: str) -> Path:
        return self.base_path / self.slug() / f"{locus}.cobs_compact"

    # ------------------------------------------------------------ training
    def fit(self, scheme_path: Path, page_size: int = DEFAULT_PAGE_SIZE) -> None:
        """One compact bank per locus directory of allele FASTA files (:101-142).

        Docs are ordered by term count then name and grouped 8*page_size per
        group; each group's signature size follows its largest doc."""
        if not scheme_path.exists():
            raise ValueError("Scheme not found. Please make sure to download the schemes prior!")
        for bank in self.indices:
            bank.close()
        self.indices, self.loci, self.avg_locus_bp_size = [], {}, []
        for locus_path in sorted(scheme_path.iterdir()):
            locus = locus_path.name
            alleles = sorted(p for p in locus_path.iterdir() if p.suffix == ".fasta")
            self.loci[locus] = len(alleles)
            self.avg_locus_bp_size.append(first_allele_length(locus_path))
            docs = []
            for p in alleles:
                seqs = [seq_text(r.seq) for r in get_record_iterator(p)]
                terms = sum(max(0, len(s) - self.k + 1) for s in seqs)
                docs.append((terms, p.stem.split(".")[0], seqs))
            docs.sort(key=lambda d: (d[0], d[1]))
            per_group = 8 * page_size
            groups = [docs[i:i + per_group] for i in range(0, len(docs), per_group)]
            sig = [cobs_signature_size(max(1, max(d[0] for d in g)), self.num_hashes, self.fpr)
                   for g in groups]
            bank = Bank.create_cobs(self.k, self.num_hashes, sig, len(docs), [d[1] for d in docs],
                                    page_size=page_size, compact=True, device=self.device)
            recs, owner = [], []
            for i, d in enumerate(docs):
                recs += d[2]
                owner += [i] * len(d[2])
            if recs:
                bank.build(pack_sequences(recs), np.asarray(owner, dtype=np.uint32))
            path = self.get_cobs_index_path(locus)
            bank.save(path)
            self.indices.append(bank)

    def save(self) -> None:
        json_path = self.base_path / f"{self.slug()}.json"
        json_path.parent.mkdir(parents=True, exist_ok=True)
        json_path.write_text(json.dumps(self.to_dict(), indent=4), encoding="utf-8")

    @staticmethod
    def load(path: Path) -> "ProbabilisticFilterMlstSchemeModel":
        if not path.exists():
            raise FileNotFoundError(f"Model JSON not found at {path}")
        meta = json.loads(path.read_text(encoding="utf-8"))
        model = ProbabilisticFilterMlstSchemeModel(
            meta["k"], meta["model_display_name"], path.parent, meta["scheme_url"],
            meta["organism"], meta["fpr"], meta["num_hashes"], meta.get("author"),
            meta.get("author_email"), meta.get("model_type"))
        model.avg_locus_bp_size = meta.get("average_locus_base_pair_size", [])
        model.loci = meta.get("loci", {})
        for locus in model.loci:
            index_path = model.get_cobs_index_path(locus)
            if not index_path.exists():
                raise FileNotFoundError(f"Index file not found at {index_path}")
            model.indices.append(Bank.open(index_path, XS_BANK_COBS_COMPACT, device=model.device))
        return model

    # ------------------------------------------------------------ helpers (reference semantics)
    def get_cobs_result(self, cobs_result, kmer_threshold: bool) -> dict:
        """{allele: score} of one result in COBS order, optionally score > 50 only (:362-380)."""
        return {r.doc_name: r.score for r in cobs_result
                if not kmer_threshold or r.score > CHUNK_KMER_THRESHOLD}

    def sequence_splitter(self, input_sequence: str, allele_len: int) -> list[str]:
        """Chunks of allele_len (x10 from 1 Mbp, x100 from 10 Mbp) overlapping by
        k-1; a tail shorter than k is appended to the last chunk (:382-426)."""
        n = len(input_sequence)
        width = allele_len if n < 1_000_000 else allele_len * 10 if n < 10_000_000 else allele_len * 100
        parts, start = [], 0
        while start + width <= n:
            parts.append(input_sequence[start:start + width])
            start += width - self.k + 1
        if start < n:
            tail = input_sequence[start:]
            if len(tail) < self.k:
                parts[-1] += tail
            else:
                parts.append(tail)
        return parts

    def has_sufficient_score(self, highest_results: dict, locus_size: list[int]) -> bool:
        """True if some locus' top score is >= half its allele length (:428-449)."""
        for i, (_, scores) in enumerate(highest_results.items()):
            if not scores:
                continue
            if next(iter(scores.values())) >= 0.5 * locus_size[i]:
                return True
        return False

    def _ordered(self, bank: Bank, row: np.ndarray, keep: np.ndarray | None = None) -> list:
        """SearchResults of one hit row in COBS order (score desc, ties by doc index)."""
        names = bank.doc_names
        idx = np.arange(row.size) if keep is None else keep
        order = idx[np.argsort(-row[idx].astype(np.int64), kind="stable")]
        return [SearchResult(names[i], int(row[i])) for i in order]

    # ------------------------------------------------------------ queries
    def _locus_rows(self, texts: list[str], step: int):
        """Per locus, one C-ABI call (xs_mlst_query) for every text: the hit
        row of each text shorter than 10 kbp, and for each longer text the
        per-allele sums of its chunk scores > 50 with the first chunk (and its
        score) that passed, computed on the device from chunk rows that never
        leave it."""
        short = [i for i, t in enumerate(texts) if len(t) < LONG_SEQUENCE]
        long_ = [i for i, t in enumerate(texts) if len(t) >= LONG_SEQUENCE]
        packed_short = pack_sequences([texts[i] for i in short])
        out = []
        for li, bank in enumerate(self.indices):
            chunks, owner = [], []
            for j, i in enumerate(long_):
                parts = self.sequence_splitter(texts[i], self.avg_locus_bp_size[li])
                chunks += parts
                owner += [j] * len(parts)
            h, sc, first, fs = bank.mlst_query(packed_short, chunks, owner, len(long_), step,
                                               CHUNK_KMER_THRESHOLD)
            rows_short = {i: h[j] for j, i in enumerate(short)}
            rows_long = {i: (sc[j], first[j], fs[j]) for j, i in enumerate(long_)}
            out.append((rows_short, rows_long))
        return out

    def _summed_counts(self, bank: Bank, summed) -> dict:
        """The reference's ``sorted_counts`` of one long text at one locus
        (:237-256): per allele the sum of its chunk scores > 50, ordered by
        -sum with ties in the order the alleles entered ``all_counts``, i.e.
        by first passing chunk, then by rank in that chunk's COBS order
        (score descending, doc index)."""
        scores, first, fscore = summed
        names = bank.doc_names
        present = np.flatnonzero(scores > 0)  # kept in some chunk (> 50 there)
        keys = (present, -fscore[present].astype(np.int64), first[present].astype(np.int64),
                -scores[present].astype(np.int64))
        order = present[np.lexsort(keys)]
        return {names[d]: int(scores[d]) for d in order}

    def _assemble(self, i: int, text: str, locus_rows, limit: bool, limit_number: int) -> list:
        scheme_loci = list(self.loci.keys())
        result_dict: dict | str = {}
        highest_results: dict = {}
        if len(text) >= LONG_SEQUENCE:
            for li, bank in enumerate(self.indices):
                sorted_counts = self._summed_counts(bank, locus_rows[li][1][i])
                if limit:
                    sorted_counts = dict(list(sorted_counts.items())[:limit_number])
                if not sorted_counts:
                    result_dict = "A Strain type could not be detected because of no kmer matches!"
                    highest_results[scheme_loci[li]] = {"N/A": 0}
                else:
                    first_key = next(iter(sorted_counts))
                    result_dict[scheme_loci[li]] = sorted_counts  # str result_dict raises, as :267
                    highest_results[scheme_loci[li]] = {first_key: sorted_counts[first_key]}
        else:
            for li, bank in enumerate(self.indices):
                result = self.get_cobs_result(self._ordered(bank, locus_rows[li][0][i]), False)
                if limit:
                    result = dict(sorted(result.items(), key=lambda x: -x[1])[:limit_number])
                result_dict[scheme_loci[li]] = result
                first_key, top = next(iter(result.items()))
                highest_results[scheme_loci[li]] = {first_key: top}
        if not self.has_sufficient_score(highest_results, self.avg_locus_bp_size):
            highest_results["Attention:"] = "This strain type is not reliable due to low kmer hit rates!"
        else:
            flattened = {locus: int(list(allele.keys())[0].split("_")[-1])
                         for locus, allele in highest_results.items()}
            resolver = self.strain_type_resolver
            highest_results["ST_Name"] = resolver(flattened, self.scheme_url) if resolver else None
        return [{"Strain type": highest_results}, {"All results": result_dict}]

    def calculate_hits(self, sequence, step: int = 1, limit: bool = False,
                       limit_number: int = 5) -> list[dict]:
        if is_record(sequence) or not isinstance(sequence, (str, bytes, bytearray)) and \
                type(sequence).__name__ not in ("Seq", "MutableSeq"):
            raise ValueError("Invalid sequence, must be a Bio.Seq object")
        text = seq_text(sequence)
        if not len(text) > self.k:
            raise ValueError("Invalid sequence, must be longer than k")
        if not self.indices:
            raise ValueError("The model has not been trained yet")
        return self._assemble(0, text, self._locus_rows([text], step), limit, limit_number)

    def predict(self, sequence_input, step: int = 1, limit: bool = False) -> MlstResult:
        """MlstResult of a record, a FASTA/FASTQ path or a record iterator (:305-360)."""
        if is_record(sequence_input):
            if sequence_input.id == "<unknown id>":
                sequence_input.id = "test"
            hits = {sequence_input.id: self.calculate_hits(sequence_input.seq, step, limit)}
            return MlstResult(self.model_display_name, step, hits, None)
        if isinstance(sequence_input, Path):
            return self.predict(get_record_iterator(sequence_input), step=step, limit=limit)
        if isinstance(sequence_input, (list, tuple, str, bytes)) or not hasattr(sequence_input, "__next__"):
            raise ValueError(
                "Invalid sequence input, must be a Seq object, a list of Seq objects, a"
                " SeqIO FastaIterator, or a SeqIO FastqPhredIterator")
        records = list(sequence_input)
        texts = [seq_text(r.seq) for r in records]
        for t in texts:
            if not len(t) > self.k:
                raise ValueError("Invalid sequence, must be longer than k")
        if not self.indices:
            raise ValueError("The model has not been trained yet")
        rows = self._locus_rows(texts, step) if texts else []
        hits = {}
        for i, rec in enumerate(records):
            hits[rec.id] = self._assemble(i, texts[i], rows, limit, 5)
        return MlstResult(self.model_display_name, step, hits, None)

    def close(self) -> None:
        for bank in self.indices:
            bank.close()
        self.indices = []
