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
  probed, exchanged) over three banks equals the C oracle's hit columns;
* configs 3 and 5 at world 2 over RCCL (two GPUs, skipped on a one-GPU box):
  child ranks started by bench.launch_ranks write shards whose merge equals
  one process's JSON byte for byte;
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


def test_predict_docs_sharded_world1_matches_oracle(pg, tmp_path, oracle_mod):
    """Config 5's library call through the device path (RCCL, world 1) for
    three banks of 40, 50 and 37 docs (127 docs in all, as three ranks of a
    multi-genus job would hold them): every bank's reads parsed on the device,
    probed, exchanged by the all-to-all; each bank's hit columns and the k-mer
    counts equal the C oracle's on the same reads, and so does the
    column-concatenated matrix one process probing every bank would write."""
    import numpy as np
    from xspect2_amd import distributed
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    banks = [_bank(oracle_mod, D=d, seed=10 + d) for d in (40, 50, 37)]
    rng = np.random.default_rng(11)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    seqs = [d[o:o + 150] for _, _, docs in banks for d in docs[::3] for o in (0, 3000)]
    seqs += [acgt[rng.integers(0, 4, int(rng.integers(22, 400)))].tobytes() for _ in range(80)]
    fa = tmp_path / "r.fasta"
    fa.write_text("".join(f">r{i} x\n{s.decode()}\n" for i, s in enumerate(seqs)))
    cols, want_cols = [], []
    for j, (ob, gb, _) in enumerate(banks):
        m = ProbabilisticFilterModel(K, f"Genus{j}", None, None, "Species", tmp_path)
        m.index = gb
        res = distributed.predict_docs_sharded(m, fa)
        want_h, want_n = ob.query(seqs)
        assert list(res.ids) == [f"r{i}" for i in range(len(seqs))]
        assert np.array_equal(res.hits.astype(np.uint32), want_h), f"bank {j}: hit columns differ from the oracle"
        assert np.array_equal(res.num_kmers.astype(np.uint64), want_n)
        cols.append(res.hits.astype(np.uint32))
        want_cols.append(want_h)
        gb.close()
    assert np.array_equal(np.concatenate(cols, axis=1), np.concatenate(want_cols, axis=1))
    assert sum(c.shape[1] for c in cols) == 127


@pytest.mark.skipif("not __import__('torch').cuda.device_count() >= 2",
                    reason="needs 2 GPUs (RCCL refuses two ranks on one device)")
def test_rccl_world2_sharded_equals_one_process(tmp_path):
    """Configs 3 and 5 over a real RCCL process group of 2 ranks (cuda:0 and
    cuda:1), each rank a fresh child process started by bench.launch_ranks
    (no GPU work in this process): classify_species_sharded (byte ranges,
    all-reduced totals, SVM label on rank 0) and predict_docs_sharded (one
    genus bank per rank, reads all-gathered, columns all-to-all'd) write
    shards whose merge is byte-equal to one process's JSON
    (tools/sharded_classify.py; src/xspect/classify.py:43-92)."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    import bench
    tool = str(root / "tools" / "sharded_classify.py")
    d = str(tmp_path)

    def one(*args):
        subprocess.run([sys.executable, tool, *args, "--root", d], check=True, timeout=600)

    one("setup", "--reads", "20000")
    one("single")
    one("docs-setup", "--world", "2", "--reads", "20000")
    one("docs-single", "--world", "2")
    env = {k: v for k, v in __import__("os").environ.items() if k != "XSPECT_SHARE_GPU"}
    for cmd in ("shard", "docs-shard"):
        assert bench.launch_ranks(2, [sys.executable, tool, cmd, "--root", d], 600, env=env) == 0
    one("check", "--world", "2")
    one("docs-check", "--world", "2")


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


def test_bench_gathers_run_on_the_device_under_rccl(pg):
    """bench.py's per-rank gathers (timings, local totals, exchange checksums)
    under an RCCL group: input and outputs on the device, results on the host
    (world 1 here; the driver's 8-GPU run takes the same call)."""
    import sys
    from pathlib import Path
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    t = torch.arange(7, dtype=torch.int64) * 3
    out = bench.all_gather_host(t, 1)
    assert len(out) == 1 and out[0].device.type == "cpu" and torch.equal(out[0], t)
    f = bench.all_gather_host(torch.tensor([1.5, 2.5], dtype=torch.float64), 1)
    assert torch.equal(f[0], torch.tensor([1.5, 2.5], dtype=torch.float64))
