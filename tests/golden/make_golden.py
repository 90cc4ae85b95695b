"""Generate the committed golden fixtures under tests/golden/.

Run here (in the build container) with:  python tests/golden/make_golden.py

Sources of truth, per fixture:
  xxh_vectors.json           python-xxhash 3.8.1 (the library XspecT imports,
                             src/xspect/models/probabilistic_single_filter_model.py:11)
  model_result_vectors.json  the reference's own ModelResult/MlstResult classes
                             (/root/reference/src/xspect/models/result.py,
                             mlst_result.py), imported read-only; only their
                             outputs are stored, never their source.
  reference_known_answers.json  data held by the reference's own tests
                             (sequences + expected numbers).
Nothing here is needed at test time except the JSON files.
"""
from __future__ import annotations

import json
import random
import sys
from pathlib import Path

import xxhash

HERE = Path(__file__).resolve().parent
REF_SRC = Path("/root/reference/src")


def xxh_vectors() -> dict:
    rng = random.Random(20260115)
    cases = []
    alph = "ACGT"
    for k in list(range(1, 65)) + [96, 127, 128, 129, 200, 240]:
        for t in range(4):
            if t == 0:
                s = "".join(rng.choice(alph) for _ in range(k)).encode()
            elif t == 1:
                s = "".join(rng.choice("ACGTNacgtnRYKM") for _ in range(k)).encode()
            else:
                s = bytes(rng.getrandbits(8) for _ in range(k))
            cases.append({
                "hex": s.hex(),
                "xxh64": [str(xxhash.xxh64_intdigest(s, seed=j)) for j in range(8)],
                "xxh3_64": str(xxhash.xxh3_64_intdigest(s)),
            })
    return {"source": f"python-xxhash {xxhash.VERSION} (libxxhash {xxhash.XXHASH_VERSION})",
            "cases": cases}


def model_result_vectors() -> dict:
    sys.path.insert(0, str(REF_SRC))
    from xspect.models.result import ModelResult  # noqa: E402  (reference, read-only)
    from xspect.models.mlst_result import MlstResult  # noqa: E402

    rng = random.Random(7)
    out = []
    for case in range(40):
        n_reads = rng.randint(1, 12)
        n_docs = rng.randint(1, 9)
        labels = [str(rng.randint(100, 99999)) for _ in range(n_docs)]
        labels = list(dict.fromkeys(labels))
        hits, nk = {}, {}
        for r in range(n_reads):
            n = rng.choice([1, 2, 3, 7, 8, 40, 60, 130, 200, 1000, rng.randint(1, 5000)])
            nk[f"read_{r}"] = n
            hits[f"read_{r}"] = {lab: rng.randint(0, n) for lab in labels}
        step = rng.choice([1, 1, 2, 3, 10])
        res = ModelResult("slug-species", {k: dict(v) for k, v in hits.items()}, dict(nk),
                          sparse_sampling_step=step, prediction=None if case % 3 else "470")
        scores = res.get_scores()
        masks = {}
        for thr in (-1, 0.0, 0.5, 0.7, 1.0):
            masks[str(thr)] = res.get_filter_mask(labels[0], thr)
        svm_vec = [v for _, v in sorted(scores["total"].items())]
        out.append({
            "hits": hits, "num_kmers": nk, "step": step,
            "prediction": None if case % 3 else "470",
            "scores": scores, "total_hits": res.get_total_hits(),
            "masks": masks,
            "filtered_07": res.get_filtered_subsequence_labels(labels[0], 0.7),
            "svm_vector": svm_vec, "to_dict": res.to_dict(),
        })
    # reference tests/test_model_result.py:6-27 known answer, stored as data
    known = ModelResult("test_slug", {"subsequence1": {"label1": 10, "label2": 5},
                                      "subsequence2": {"label1": 8, "label2": 3}},
                        {"subsequence1": 100, "subsequence2": 50})
    mlst = MlstResult("Oxford", 1, {"test": [{"Strain type": {"Oxf_cpn60": {"Allele_ID_4": 401}}},
                                             {"All results": {}}]}, "in.fasta")
    return {"source": "reference result.py / mlst_result.py imported from /root/reference",
            "cases": out, "known_get_scores": known.get_scores(),
            "mlst_to_dict": mlst.to_dict()}


def reference_known_answers() -> dict:
    # Data held by the reference's own tests (not their source).
    return {
        "salmonella_80bp": {
            "seq": "AGAGATTACGTCTGGTTGCAAGAGATCATGACAGGGGGAATTGGTTGAAAATAAATATATCGCCAGCAGCACATGAACAA",
            "k": 21, "num_kmers": 60, "hits_self_by_step": {"1": 60, "2": 30, "3": 20, "4": 15},
            "source": "tests/test_probabilistic_filter_model.py:139-161",
        },
        "splitter": {
            "seq": "AGCTATTTCGCTGATGTCGACTGATCAAAAAGCCGGCGCGCTTTCGTATAGGCTAGCTACGACATACGATCGATCACTGA",
            "k": 4, "allele_len": 20, "num_parts": 5,
            "source": "tests/test_probabilistic_filter_mlst_model.py:127-142",
        },
        "genus_query": {
            "seq": "TAAATAAATTTATATAGCTAAA", "k": 21, "num_kmers": 2, "hits_if_all_present": 2,
            "source": "tests/test_probabilistic_single_filter_model.py:42-45",
        },
        "cpn60_allele4": {
            "seq": ("ATGAACCCAATGGATTTAAAACGCGGTATCGACATTGCAGTAAAAACTGTAGTTGAAAAT"
                    "ATCCGTTCTATTGCTAAACCAGCTGATGATTTCAAAGCAATTGAACAAGTAGGTTCAATC"
                    "TCTGCTAACTCTGATACTACTGTTGGTAAACTTATTGCTCAAGCAATGGAAAAAGTAGGT"
                    "AAAGAAGGCGTAATCACTGTAGAAGAAGGTTCTGGCTTCGAAGACGCATTAGACGTTGTA"
                    "GAAGGTATGCAGTTTGACCGTGGTTATATCTCTCCGTACTTTGCAAACAAACAAGATACT"
                    "TTAACTGCTGAACTTGAAAATCCGTTCATTCTTCTTGTTGATAAAAAAATCAGCAACATT"
                    "CGTGAATTGATTTCTGTTTTAGAAGCAGTTGCTAAAACTGGTAAACCACTTCTTATCATC"
                    "G"),
            "k": 21, "self_score": 401,
            "source": "tests/test_probabilistic_filter_mlst_model.py:82-99",
        },
    }


def main() -> None:
    for name, fn in [("xxh_vectors.json", xxh_vectors),
                     ("model_result_vectors.json", model_result_vectors),
                     ("reference_known_answers.json", reference_known_answers)]:
        (HERE / name).write_text(json.dumps(fn(), indent=1, sort_keys=False))
        print("wrote", name)


if __name__ == "__main__":
    main()
