"""Config 3 rehearsal: `classify species` sharded over ranks vs one process.

    python tools/sharded_classify.py setup  --root DIR [--reads N]   # model (GPU fit) + reads.fq
    python tools/sharded_classify.py single --root DIR               # classify_species -> single.json
    torchrun --nproc-per-node N tools/sharded_classify.py shard --root DIR
    python tools/sharded_classify.py check  --root DIR --world N     # merged shards == single.json

Config 5 (docs sharded; one genus model per rank; rank r parses its byte
range, the reads are all-gathered, the hit columns go back to their reads'
rank by all-to-all, every rank writes its shard):
    python tools/sharded_classify.py docs-setup  --root DIR --world N [--reads R]  # N genus models of 60 species
    python tools/sharded_classify.py docs-single --root DIR --world N              # all models in one process
    torchrun --nproc-per-node N tools/sharded_classify.py docs-shard --root DIR
    python tools/sharded_classify.py docs-check  --root DIR --world N

Config 5 with ONE bank column-split over the ranks (the `setup` model):
    python tools/sharded_classify.py bank-single --root DIR        # predict_columnar -> bank_single.json
    torchrun --nproc-per-node N tools/sharded_classify.py bank-shard --root DIR
    python tools/sharded_classify.py bank-check  --root DIR --world N

`shard` runs xspect2_amd.classify.classify_species_sharded: each rank parses
its byte range of reads.fq, the D+1 totals are all-reduced (RCCL, or gloo
with XSPECT_SHARE_GPU=1 when the ranks share one GPU), rank 0 forms the SVM
label, every rank writes its JSON shard.  Each step is its own process.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
GENUS = "Acinetobacter"
GENERA = ["Acinetobacter", "Pseudomonas", "Klebsiella", "Escherichia", "Salmonella", "Enterobacter",
          "Staphylococcus", "Streptococcus"]


def setup(root: Path, n_reads: int, dup: bool = False) -> None:
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
    from xspect2_amd.synth import make_genomes, make_reads
    from xspect2_amd.file_io import Record, write_fasta

    os.environ["XSPECT_DATA"] = str(root / "xspect-data")
    genomes = make_genomes(12, 200_000, seed=42)
    sp = root / "species"
    svm = root / "svm"
    for d in range(12):
        g = genomes[d].tobytes().decode()
        write_fasta([Record(f"c{d}", g[:150_000])], sp / f"GCF_{470 + 31 * d:09d}.1_genomic.fna", width=80)
        for j in range(2):
            write_fasta([Record("x", g[100_000 + 40_000 * j:140_000 + 40_000 * j])],
                        svm / f"label{d:02d}" / f"acc{d}{j}.fasta")
    model = ProbabilisticFilterSVMModel(21, GENUS, None, None, "Species", root / "xspect-data" / "models", "rbf", 1.0)
    model.fit(sp, svm, svm_step=50)
    model.save()
    reads, _ = make_reads(genomes, n_reads, 150, seed=43)
    with open(root / "reads.fq", "w") as fh:
        for i in range(n_reads):
            s = reads[i].tobytes().decode()
            rid = i % (n_reads // 2) if dup else i  # dup: read i and i + n/2 share an id (different shards)
            fh.write(f"@read_{rid} synthetic\n{s}\n+\n{'I' * len(s)}\n")


def docs_setup(root: Path, n_reads: int, world: int) -> None:
    """`world` genus species models of 60 species each (fit on the GPU) and reads from all their genomes."""
    import numpy as np
    from xspect2_amd.file_io import Record, write_fasta
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    from xspect2_amd.synth import make_genomes, make_reads

    allg = []
    for gi, genus in enumerate(GENERA[:world]):
        genomes = make_genomes(60, 100_000, seed=100 + gi)
        allg.append(genomes)
        sp = root / f"species_{genus}"
        for d in range(60):
            write_fasta([Record(f"c{d}", genomes[d].tobytes().decode())], sp / f"GCF_{1000 * (gi + 1) + d:09d}.fna")
        model = ProbabilisticFilterModel(21, genus, None, None, "Species", root / "xspect-data" / "models")
        model.fit(sp)
        model.save()
    reads, _ = make_reads(np.concatenate(allg), n_reads, 150, seed=44)
    with open(root / "docs_reads.fasta", "w") as fh:
        for i in range(n_reads):
            fh.write(f">dread_{i}\n{reads[i].tobytes().decode()}\n")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["setup", "single", "shard", "check", "docs-setup", "docs-single", "docs-shard",
                                    "docs-check", "bank-single", "bank-shard", "bank-check"])
    ap.add_argument("--root", required=True)
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--dup", action="store_true", help="setup: every read id occurs twice, n/2 records apart")
    a = ap.parse_args()
    root = Path(a.root).resolve()
    root.mkdir(parents=True, exist_ok=True)
    os.environ["XSPECT_DATA"] = str(root / "xspect-data")
    t0 = time.time()
    if a.cmd == "setup":
        setup(root, a.reads, a.dup)
    elif a.cmd == "single":
        from xspect2_amd import classify
        classify.classify_species(GENUS, root / "reads.fq", root / "single.json", step=a.step)
    elif a.cmd == "shard":
        import torch
        import torch.distributed as dist
        from xspect2_amd import classify
        share = os.environ.get("XSPECT_SHARE_GPU") == "1"
        local = 0 if share else int(os.environ.get("LOCAL_RANK", "0"))
        os.environ["XSPECT2_AMD_DEVICE"] = str(local)
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        classify.classify_species_sharded(GENUS, root / "reads.fq", root / "sharded.json", step=a.step)
        dist.barrier()
        dist.destroy_process_group()
    elif a.cmd == "docs-setup":
        docs_setup(root, a.reads, a.world)
    elif a.cmd == "docs-single":
        import numpy as np
        from xspect2_amd import classify
        from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
        from xspect2_amd.result import MatrixResult
        parts = [ProbabilisticFilterModel.load(classify.species_model_path(g)).predict_columnar(
            root / "docs_reads.fasta", step=a.step) for g in GENERA[:a.world]]
        hits = np.concatenate([p.hits.astype(np.uint32) for p in parts], axis=1)
        res = MatrixResult("multi-genus-docs-sharded", parts[0].ids, [lab for p in parts for lab in p.labels], hits,
                           parts[0].num_kmers, sparse_sampling_step=a.step)
        res.input_source = "docs_reads.fasta"
        res.save(root / "docs_single.json")
    elif a.cmd == "docs-shard":
        import torch
        import torch.distributed as dist
        from xspect2_amd import classify, distributed
        from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
        share = os.environ.get("XSPECT_SHARE_GPU") == "1"
        local = 0 if share else int(os.environ.get("LOCAL_RANK", "0"))
        os.environ["XSPECT2_AMD_DEVICE"] = str(local)
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        model = ProbabilisticFilterModel.load(classify.species_model_path(GENERA[dist.get_rank()]))
        # each rank writes the shard of its own reads (byte range of the file)
        distributed.classify_docs_sharded(model, root / "docs_reads.fasta", root / "docs_sharded.json", step=a.step)
        dist.barrier()
        dist.destroy_process_group()
    elif a.cmd == "bank-single":
        from xspect2_amd import classify
        from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
        res = ProbabilisticFilterSVMModel.load(classify.species_model_path(GENUS)).predict_columnar(
            root / "reads.fq", step=a.step)
        res.input_source = "reads.fq"
        res.save(root / "bank_single.json")
    elif a.cmd == "bank-shard":
        import torch
        import torch.distributed as dist
        from xspect2_amd import classify, distributed
        from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
        share = os.environ.get("XSPECT_SHARE_GPU") == "1"
        local = 0 if share else int(os.environ.get("LOCAL_RANK", "0"))
        os.environ["XSPECT2_AMD_DEVICE"] = str(local)
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        model = distributed.load_docs_slice(ProbabilisticFilterSVMModel, classify.species_model_path(GENUS))
        print(f"rank {dist.get_rank()}: docs {model.index.num_docs}", file=sys.stderr)
        res = distributed.predict_bank_sharded(model, root / "reads.fq", step=a.step)
        res.save(distributed.shard_path(root / "bank_sharded.json", dist.get_rank(), dist.get_world_size()))
        dist.barrier()
        dist.destroy_process_group()
    else:  # check, docs-check, bank-check: the shards streamed into one file (merge_result_files) vs one process's
        from xspect2_amd.distributed import merge_result_files, shard_path
        stem = {"check": ("single", "sharded"), "docs-check": ("docs_single", "docs_sharded"),
                "bank-check": ("bank_single", "bank_sharded")}[a.cmd]
        shards = [shard_path(root / f"{stem[1]}.json", r, a.world) for r in range(a.world)]
        merge_result_files(shards, root / f"{stem[1]}_merged.json")
        a_ = (root / f"{stem[0]}.json").read_bytes()
        b_ = (root / f"{stem[1]}_merged.json").read_bytes()
        # per-shard read counts from the shards' num_kmers sections (cheap: one line per read)
        per = []
        for p in shards:
            t = p.read_bytes()
            i = t.find(b'"num_kmers": ')
            per.append(t[i:t.find(b'"misclassified"', i)].count(b"\n        "))
        print(json.dumps({"world": a.world, "equal_bytes": a_ == b_, "json_bytes": len(a_), "reads_per_shard": per,
                          "reads": sum(per)}))
        return 0 if a_ == b_ else 1
    print(f"{a.cmd}: {time.time() - t0:.1f}s", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
