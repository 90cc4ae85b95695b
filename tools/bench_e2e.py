"""End-to-end file -> hits timing of the species path.

Writes a synthetic FASTQ of --reads x 150 bp reads (seeded genomes of the
bench's config-2 bank), then times:
  parse      native reader alone (xs_fastx_next over the whole file)
  dparse     the reader's device mode alone (text -> HBM, records found on the GPU)
  e2e_dev_*  the same streaming with the device-mode reader (DeviceSeqBatch ->
             xs_query_hits_device): min over --reps passes, and the first pass
  e2e        ProbabilisticFilterModel-style streaming: read_batches -> Bank.query
             (H2D, probe, D2H of the n x D hit matrix), parse overlapped
  e2e_tot    same, but per-doc totals only (xs_query_totals, no hit matrix)
  e2e_best   read_batches -> Bank.query_best (per-read best doc on the device)
  classify   ProbabilisticFilterModel.predict_columnar(file) + MatrixResult.save of
             the whole file (the product's classify path, device-mode reader)
  json       MatrixResult.save (native writer) of the first 200k reads' result, and
             the per-read-dict ModelResult.save on a 20k-read sample, scaled
  py_parse   the pure-Python restatement of Bio.SeqIO (oracle/fastx.py) on a
             bounded sample, scaled: what a record-at-a-time host path costs
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--docs", type=int, default=100)
    ap.add_argument("--genome-len", type=int, default=4_000_000)
    ap.add_argument("--batch-mb", type=int, default=256)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--quick", action="store_true", help="parse and e2e legs only")
    ap.add_argument("--profile-classify", default=None,
                    help="write a cProfile summary of a second predict_columnar(file) to this path")
    args = ap.parse_args()

    import torch
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.file_io import FastxReader, read_batches
    from xspect2_amd.synth import make_genomes, make_reads

    k = 21
    dev = torch.device("cuda", 0)
    genomes = make_genomes(args.docs, args.genome_len, seed=42)
    sig = cobs_signature_size(args.genome_len - k + 1, 7, 0.01)
    bank = Bank.create_cobs(k, 7, [sig], args.docs, [f"sp{i:03d}" for i in range(args.docs)], device=0)
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(args.docs + 1, dtype=torch.int64, device=dev) * args.genome_len
    bank.build_device(g, genomes.size, go, args.docs, torch.arange(args.docs, dtype=torch.int32, device=dev),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del g

    reads, _ = make_reads(genomes, args.reads, 150, seed=42)
    tmp = Path(args.dir or tempfile.mkdtemp(prefix="xs_e2e_"))
    tmp.mkdir(parents=True, exist_ok=True)
    fq = tmp / "reads.fastq"
    qual = b"I" * 150
    with open(fq, "wb") as fh:
        for i in range(reads.shape[0]):
            fh.write(b"@r%d\n%s\n+\n%s\n" % (i, reads[i].tobytes(), qual))
    size = fq.stat().st_size
    mb = args.batch_mb << 20
    res = {"file_bytes": size, "reads": int(reads.shape[0]), "docs": args.docs, "batch_mb": args.batch_mb}

    # parse only
    t = time.perf_counter()
    n = 0
    with FastxReader(fq) as rd:
        for b in rd.batches(mb):
            n += b.n
    dt = time.perf_counter() - t
    assert n == reads.shape[0]
    res["parse_s"] = dt
    res["parse_GBps"] = size / dt / 1e9

    # device-mode reader: parse only, then file -> hits / totals
    def timed(fn):
        ts = []
        for _ in range(max(1, args.reps)):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return min(ts), ts[0]

    def dparse():
        n_ = 0
        on_dev = True
        for b in read_batches(fq, mb, device=0):
            n_ += b.n
            on_dev &= b.parsed_on_device
        assert n_ == reads.shape[0] and on_dev
    res["dparse_s"], res["dparse_first_s"] = timed(dparse)
    res["dparse_GBps"] = size / res["dparse_s"] / 1e9
    print("dparse", res["dparse_s"], file=sys.stderr, flush=True)
    from xspect2_amd.file_io import FastxReader
    with FastxReader(fq, device=0) as rdd, FastxReader(fq) as rdh:  # batches live as long as their readers
        first_dev, first_host = rdd.next_batch(mb), rdh.next_batch(mb)
        hd, nd = bank.query(first_dev, hit_dtype="auto")
        hh, nh = bank.query(first_host.packed, hit_dtype="auto")
        res["device_reader_first_batch_equal"] = bool(np.array_equal(hd, hh) and np.array_equal(nd, nh)
                                                      and first_dev.ids() == first_host.ids())
    del first_dev, first_host
    from xspect2_amd.bank import pinned_empty as _pe
    dev_sizes = [b.n for b in read_batches(fq, mb, device=0)]
    dev_outs = {n_: _pe((n_, args.docs), np.uint8) for n_ in set(dev_sizes)}
    for name, fn in (("hits_auto", lambda b: bank.query(b, hit_dtype="auto")),
                     ("hits_u8_pinned_out", lambda b: bank.query(b, hit_dtype=np.uint8, out=dev_outs[b.n])),
                     ("totals", lambda b: bank.query_totals(b))):
        def run(fn=fn):
            for b in read_batches(fq, mb, device=0):
                fn(b)
        res[f"e2e_dev_{name}_s"], res[f"e2e_dev_{name}_first_s"] = timed(run)
        res[f"e2e_dev_{name}_reads_per_s"] = reads.shape[0] / res[f"e2e_dev_{name}_s"]
        print(name, res[f"e2e_dev_{name}_s"], file=sys.stderr, flush=True)
    if args.quick:
        for pinned in (False, True):
            t = time.perf_counter()
            for b in read_batches(fq, mb, pinned=pinned):
                bank.query(b.packed, hit_dtype="auto")
            res[f"e2e_hits_auto_s{'_pinned' if pinned else ''}"] = time.perf_counter() - t
        print(json.dumps(res))
        return

    for pinned in (False, True):
        # warm
        for b in read_batches(fq, mb, pinned=pinned):
            bank.query(b.packed)
            break
        t = time.perf_counter()
        n = 0
        for b in read_batches(fq, mb, pinned=pinned):
            h, nk = bank.query(b.packed)
            n += b.n
        dt = time.perf_counter() - t
        res[f"e2e_hits_s{'_pinned' if pinned else ''}"] = dt
        res[f"e2e_hits_reads_per_s{'_pinned' if pinned else ''}"] = n / dt
        t = time.perf_counter()
        for b in read_batches(fq, mb, pinned=pinned):
            bank.query_totals(b.packed)
        dt = time.perf_counter() - t
        res[f"e2e_totals_s{'_pinned' if pinned else ''}"] = dt
        res[f"e2e_totals_reads_per_s{'_pinned' if pinned else ''}"] = n / dt

    # the model path since round 3 (Bank.query(hit_dtype="auto")): the hit
    # matrix narrowed on the device (u8 for 150 bp reads) into fresh pageable
    # arrays; and the same into pinned buffers a serving loop reuses
    from xspect2_amd.bank import pinned_empty
    sizes = [b.n for b in read_batches(fq, mb)]
    outs = {n_: pinned_empty((n_, args.docs), np.uint8) for n_ in set(sizes)}
    for name, kw in (("auto", lambda b: {"hit_dtype": "auto"}),
                     ("u8_pinned_out", lambda b: {"hit_dtype": np.uint8, "out": outs[b.n]})):
        t = time.perf_counter()
        n = 0
        for b in read_batches(fq, mb, pinned=True):
            h, nk = bank.query(b.packed, **kw(b))
            n += b.n
        dt = time.perf_counter() - t
        res[f"e2e_hits_{name}_s"] = dt
        res[f"e2e_hits_{name}_reads_per_s"] = n / dt

    # per-read best doc, hit matrix kept on the device
    t = time.perf_counter()
    n = 0
    for b in read_batches(fq, mb, pinned=True):
        best, bh, nk, tot = bank.query_best(b.packed, want_totals=True)
        n += b.n
    dt = time.perf_counter() - t
    res["e2e_best_s_pinned"] = dt
    res["e2e_best_reads_per_s_pinned"] = n / dt

    # result JSON: columnar writer (whole file) vs per-read dicts (sample, scaled)
    from xspect2_amd.result import MatrixResult
    ids, hs, nks = [], [], []
    for b in read_batches(fq, mb):
        h, nk = bank.query(b.packed, hit_dtype="auto")
        ids += b.ids()
        hs.append(h)
        nks.append(nk)
    hits = np.concatenate(hs)
    nk = np.concatenate(nks)
    labels = bank.doc_names
    J = min(len(ids), 200_000)  # ~1 GB of JSON
    mr = MatrixResult("synthetic-species", ids[:J], labels, hits[:J], nk[:J], input_source=fq.name)
    out = tmp / "result.json"
    t = time.perf_counter()
    mr.save(out)
    dt = time.perf_counter() - t
    res["json_reads"] = J
    res["json_columnar_s"] = dt
    res["json_bytes"] = out.stat().st_size
    res["json_columnar_MBps"] = out.stat().st_size / dt / 1e6
    m = 20_000
    small = MatrixResult("synthetic-species", ids[:m], labels, hits[:m], nk[:m], input_source=fq.name)
    t = time.perf_counter()
    small.to_model_result().save(tmp / "small_dicts.json")
    dt = time.perf_counter() - t
    res["json_dicts_s_scaled"] = dt * J / m
    small.save(tmp / "small_columnar.json")
    res["json_small_identical"] = (tmp / "small_dicts.json").read_bytes() == (tmp / "small_columnar.json").read_bytes()
    for f in (out, tmp / "small_dicts.json", tmp / "small_columnar.json"):
        f.unlink()

    # fused genus -> species pipeline vs the reference's three passes, on 200k reads
    from xspect2_amd.bank import bloom_parameters
    from xspect2_amd.pipeline import reference_pipeline, run_pipeline
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    from xspect2_amd.probabilistic_single_filter_model import ProbabilisticSingleFilterModel
    half = args.docs // 2  # the genus filter holds half of the species: about half of the reads pass
    gsz = genomes[:half].size
    nb, nh = bloom_parameters(gsz - k + 1, 0.01)
    gbank = Bank.create_bloom(k, nb, nh, device=0)
    g = torch.from_numpy(genomes[:half].reshape(-1)).to(dev)
    go = torch.arange(half + 1, dtype=torch.int64, device=dev) * args.genome_len
    gbank.build_device(g, gsz, go, half, None, stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    genus = ProbabilisticSingleFilterModel(k, "Synthetic", None, None, "Genus", tmp / "models")
    genus.bf = genus.index = gbank
    genus.display_names = {"Synthetic": "Synthetic"}
    species = ProbabilisticFilterModel(k, "Synthetic", None, None, "Species", tmp / "models")
    species.index = bank
    species.display_names = {nm: nm for nm in bank.doc_names}
    R = min(reads.shape[0], 200_000)
    sub = tmp / "sub.fastq"
    with open(sub, "wb") as fh:
        for i in range(R):
            fh.write(b"@r%d\n%s\n+\n%s\n" % (i, reads[i].tobytes(), qual))
    quiet = lambda *a: None  # noqa: E731
    t = time.perf_counter()
    outf = run_pipeline(genus, species, sub, tmp / "fused", threshold=0.7, run_id="x", log=quiet)
    res["pipeline_fused_s"] = time.perf_counter() - t
    t = time.perf_counter()
    outr = reference_pipeline(genus, species, sub, tmp / "three_pass", threshold=0.7, run_id="x", log=quiet)
    res["pipeline_three_pass_s"] = time.perf_counter() - t
    res["pipeline_reads"] = R
    res["pipeline_kept_reads"] = outf["filtered"][0].read_bytes().count(b">") if outf["filtered"] else 0
    res["pipeline_identical"] = all(a.read_bytes() == b.read_bytes() for key in ("genus", "filtered", "species")
                                    for a, b in zip(outf[key], outr[key]))
    # the product's classify path on the whole file: predict_columnar (device-mode
    # reader, narrow hit rows back) then MatrixResult.save (the reference's JSON)
    t = time.perf_counter()
    cres = species.predict_columnar(fq)
    res["classify_predict_s"] = time.perf_counter() - t
    cres.input_source = fq.name
    if args.profile_classify:  # where the host side of predict_columnar goes (warm)
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        t = time.perf_counter()
        pr.enable()
        species.predict_columnar(fq)
        pr.disable()
        res["classify_predict_again_s"] = time.perf_counter() - t
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(30)
        Path(args.profile_classify).write_text(buf.getvalue())
    t = time.perf_counter()
    cres.save(tmp / "classify.json")
    res["classify_save_s"] = time.perf_counter() - t
    res["classify_json_bytes"] = (tmp / "classify.json").stat().st_size
    res["classify_reads"] = len(cres.ids)
    (tmp / "classify.json").unlink()
    del cres
    import shutil
    shutil.rmtree(tmp / "fused")
    shutil.rmtree(tmp / "three_pass")
    sub.unlink()

    # record-at-a-time Python parse on a bounded sample, scaled to the file
    sys.path.insert(0, str(ROOT / "oracle"))
    import fastx as ofx  # test/bench-only restatement of Bio.SeqIO
    sample = fq.read_bytes()[: 40 << 20]
    sample = sample[: sample.rfind(b"\n@") + 1]
    t = time.perf_counter()
    recs = ofx.parse_fastq(sample)
    dt = time.perf_counter() - t
    res["py_parse_sample_bytes"] = len(sample)
    res["py_parse_GBps"] = len(sample) / dt / 1e9
    res["py_parse_s_scaled"] = dt * size / len(sample)
    res["py_parse_records"] = len(recs)

    # hits agree with the packed-in-memory path on the first batch
    with FastxReader(fq) as rd:
        b = rd.next_batch(mb)
        h1, _ = bank.query(b.packed)
    from xspect2_amd.packing import pack_fixed
    h2, _ = bank.query(pack_fixed(reads[: b.n]))
    res["first_batch_hits_equal"] = bool(np.array_equal(h1, h2))
    print(json.dumps(res))
    if not args.dir:
        fq.unlink()


if __name__ == "__main__":
    main()
