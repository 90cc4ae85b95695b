"""The device-resident multi-GPU paths on one MI355X (GPU), in a world-1 RCCL
process group: the collectives run on device tensors exactly as at N = 8,
with one participant.  (Multi-rank equality is tested with gloo on the CPU,
tests/test_distributed_sharded.py, and rehearsed with torchrun on the GPU box
by tools/gpu/gpu_r03_sharded.sh.)

* config 5: ``docs_sharded_hits_device`` — probe on the device, narrow, RCCL
  all-gather, widen — equals the bank's hit matrix, for 1-byte and 2-byte
  transport; ``exchange_doc_columns`` (the all-to-all that sends every
  rank's hit columns to the reads' rank) keeps values in 1, 2 and 4 bytes;
  ``predict_docs_sharded`` (reads all-gathered from the device reader,
  probed, exchanged) equals the model's own prediction;
* config 3: ``classify_species_sharded`` — the byte-range reader, the RCCL
  all-reduce of D+1 totals on a device tensor, the SVM label — writes the
  JSON the single-process ``classify_species`` writes.
"""
from __future__ import annotations

import json
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 21


@pytest.fixture(scope="module")
def pg():
    import torch
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


def _bank(oracle_mod, D=100, seed=0):
    from xspect2_amd.bank import Bank
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    docs = [acgt[rng.integers(0, 4, 5000)].tobytes() for _ in range(D)]
    sig = [oracle_mod.signature_size(5000, 7, 0.01)]
    ob = oracle_mod.CobsBank.empty(sig, (D + 7) // 8, D, 7, K)
    ob.build(docs, list(range(D)))
    gb = Bank.create_cobs(K, 7, sig, D, [f"s{i}" for i in range(D)])
    gb.upload(ob.rows)
    return ob, gb, docs


@pytest.mark.parametrize("read_len,wire", [(150, "uint8"), (2000, "int16")])
def test_docs_sharded_gather_on_device(pg, oracle_mod, read_len, wire):
    import torch
    from xspect2_amd import distributed
    from xspect2_amd.packing import pack_sequences
    ob, gb, docs = _bank(oracle_mod)
    rng = np.random.default_rng(read_len)
    reads = [d[o:o + read_len] for d in docs[:60] for o in (0, 1000, 2500)]
    reads += [np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, read_len)].tobytes() for _ in range(40)]
    pr = pack_sequences(reads)
    dev = torch.device("cuda", 0)
    d_seq = torch.from_numpy(pr.buf.copy()).to(dev)
    d_off = torch.from_numpy(pr.offsets.astype(np.int64)).to(dev)
    hits, nk = distributed.docs_sharded_hits_device(gb, d_seq, pr.nbytes, d_off, pr.n, 1)
    assert hits.is_cuda and hits.dtype == torch.int32 and tuple(hits.shape) == (pr.n, 100)
    want, want_n = ob.query(reads)
    assert np.array_equal(hits.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(nk.cpu().numpy().view(np.uint64), want_n)
    dims, dt = distributed.doc_shard_layout(100, int(want_n.max()))
    assert dims == [100] and str(dt) == f"torch.{wire}"
    gb.close()


def test_classify_species_sharded_world1_equals_classify_species(pg, tmp_path, monkeypatch):
    from xspect2_amd import classify, distributed
    from xspect2_amd.file_io import Record, write_fasta
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
    from xspect2_amd.synth import make_genomes, make_reads

    root = tmp_path / "xspect-data"
    monkeypatch.setenv("XSPECT_DATA", str(root))
    genomes = make_genomes(5, 40_000, seed=3)
    for d in range(5):
        g = genomes[d].tobytes().decode()
        write_fasta([Record(f"c{d}", g[:30_000])], tmp_path / "sp" / f"GCF_{900 + d:09d}.1_x.fna")
        for j in range(2):
            write_fasta([Record("x", g[20_000 + 8000 * j:30_000 + 8000 * j])], tmp_path / "svm" / f"L{d}" / f"a{j}.fasta")
    model = ProbabilisticFilterSVMModel(K, "Acinetobacter", None, None, "Species", root / "models", "rbf", 1.0)
    model.fit(tmp_path / "sp", tmp_path / "svm", svm_step=10)
    model.save()
    reads, _ = make_reads(genomes, 3000, 150, seed=5)
    fq = tmp_path / "reads.fq"
    fq.write_text("".join(f"@r{i}\n{reads[i].tobytes().decode()}\n+\n{'I' * 150}\n" for i in range(3000)))
    classify.classify_species("Acinetobacter", fq, tmp_path / "single.json", step=2)
    outs = classify.classify_species_sharded("Acinetobacter", fq, tmp_path / "sharded.json", step=2)
    assert outs == [tmp_path / "sharded.json"]
    shard = distributed.shard_path(tmp_path / "sharded.json", 0, 1)
    want = json.loads((tmp_path / "single.json").read_text())
    assert distributed.merge_result_shards([shard]) == want
    assert shard.read_bytes() == (tmp_path / "single.json").read_bytes()  # one shard = the whole file
    assert want["prediction"].startswith("L")


def test_predict_docs_sharded_world1_on_device(pg, tmp_path, oracle_mod):
    """Config 5's library call through the device path (RCCL, world 1):
    equals the model's own columnar prediction."""
    import numpy as np
    from xspect2_amd import distributed
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    ob, gb, docs = _bank(oracle_mod, D=100, seed=3)
    m = ProbabilisticFilterModel(K, "Genus", None, None, "Species", tmp_path)
    m.index = gb
    fa = tmp_path / "r.fasta"
    fa.write_text("".join(f">r{i}\n{d[o:o + 150].decode()}\n" for i, d in enumerate(docs) for o in (0, 3000)))
    res = distributed.predict_docs_sharded(m, fa)
    want = m.predict_columnar(fa)
    assert res.ids == want.ids and res.labels == want.labels
    assert np.array_equal(res.hits.astype(np.uint32), want.hits.astype(np.uint32))
    assert np.array_equal(res.num_kmers, want.num_kmers)
    gb.close()


@pytest.mark.parametrize("wire", ["uint8", "int16", "int32"])
def test_exchange_doc_columns_on_device(pg, wire):
    """Config 5's output exchange (RCCL all-to-all, world 1): the rank's hit
    columns come back narrowed to the wire type, values intact (int16 rides
    as float16 bit patterns)."""
    import torch
    from xspect2_amd import distributed
    dt = getattr(torch, wire)
    top = {"uint8": 255, "int16": 32767, "int32": 1 << 30}[wire]
    g = torch.Generator(device="cuda").manual_seed(5)
    hits = torch.randint(0, top + 1, (3001, 37), generator=g, device="cuda", dtype=torch.int64).to(torch.int32)
    out = distributed.exchange_doc_columns(hits, [3001], [37], dt)
    assert out.dtype == dt and out.device == hits.device and tuple(out.shape) == (3001, 37)
    assert torch.equal(out.to(torch.int64), hits.to(torch.int64))
