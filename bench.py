"""Throughput of the k-mer x filter probe path on MI355X (driver contract).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Workload (BASELINE.json configs[1]): 1M synthetic
150 bp reads per GPU against a D=100 species COBS classic bank (k=21, h=7,
fpr=0.01; ~38M rows, 0.5 GB file / 0.6 GB in HBM, larger than the 256 MiB
Infinity Cache).  One step = one query of the whole read batch, resident in
HBM: strands -> units -> probe -> totals; with N>1 ranks the per-doc totals
(D+1 uint64, the input of the SVM vector) are all-reduced over RCCL.  Reads
are sharded (seed 42+rank), the bank is replicated: weak scaling.

metric = k-mer x filter probes / s = sum(ceil((L-k+1)/step)) * D / seconds,
whole job.  The roofline entry prices the probe kernel alone (HIP events on
its launch stream, every step of the timed region) at its algorithmic bytes:
h x 64 B per k-mer (one random row transaction per hash) + the streamed
strand windows, hit matrix and per-read metadata; peak = 8.0 TB/s HBM3E.
cpu_baseline: the C oracle (oracle/liboracle.so, OpenMP) on a bounded sample
of the same reads and bank, rank 0 only, N=1 only; its hits are also checked
bit-exact against the GPU hits of the same reads.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0
ROW_BYTES = 64  # one random HBM transaction per signature row


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=1_000_000, help="reads per GPU")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--docs", type=int, default=100)
    ap.add_argument("--genome-len", type=int, default=4_000_000)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--hashes", type=int, default=7)
    ap.add_argument("--fpr", type=float, default=0.01)
    ap.add_argument("--step", type=int, default=1, help="sparse sampling step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic_r01.json"))
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from xspect_amd.bank import Bank, cobs_signature_size
    from xspect_amd.synth import make_genomes, make_reads

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    k, h, D = args.k, args.hashes, args.docs
    t_setup = time.time()
    genomes = make_genomes(D, args.genome_len, seed=42)
    sig = cobs_signature_size(args.genome_len - k + 1, h, args.fpr)
    names = [f"species_{i:03d}" for i in range(D)]
    bank = Bank.create_cobs(k, h, [sig], D, names, device=local)
    g_dev = torch.from_numpy(genomes.reshape(-1)).to(dev)
    g_offs = torch.arange(D + 1, dtype=torch.int64, device=dev) * args.genome_len
    g_docs = torch.arange(D, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    bank.build_device(g_dev, genomes.size, g_offs, D, g_docs, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    del g_dev
    info = bank.info
    log(rank, f"bank: D={D} k={k} h={h} S={sig} rows, {info.device_bytes / 1e9:.2f} GB in HBM "
              f"(built in {time.time() - t_setup:.1f}s incl. genomes)")

    reads, _ = make_reads(genomes, args.reads, args.read_len, seed=42 + rank)
    n = reads.shape[0]
    seq_bytes = reads.size
    d_seqs = torch.from_numpy(reads.reshape(-1)).to(dev)
    d_offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * args.read_len
    d_hits = torch.empty((n, D), dtype=torch.int32, device=dev)
    d_nk = torch.empty(n, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(D + 1, dtype=torch.int64, device=dev)
    nk_read = (args.read_len - k + args.step) // args.step
    kmers_per_rank = n * nk_read

    def step():
        bank.query_device(d_seqs, seq_bytes, d_offs, n, args.step, d_hits, d_nk, d_tot,
                          stream=stream.cuda_stream)
        if world > 1:
            dist.all_reduce(d_tot)  # RCCL: per-doc totals + k-mer total over all ranks

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    bank.set_profiling(True)
    bank.probe_stats()  # reset
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    bank.set_profiling(False)
    launches, probe_ms_total, probe_ms_max = bank.probe_stats()
    probe_ms = probe_ms_total / max(1, launches)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity of the last step (whole-job totals)
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert int(tot[D]) == kmers_per_rank * world, "k-mer total mismatch"

    probes = kmers_per_rank * world * D
    value = probes * args.steps / elapsed
    algo_bytes = (kmers_per_rank * h * ROW_BYTES      # random row transactions
                  + 2 * seq_bytes                     # forward + reverse-complement windows
                  + n * D * 4                         # hit matrix
                  + n * (8 + 4 + 8 + 8))              # offsets, unit map, unit offsets, num_kmers
    achieved = algo_bytes / (probe_ms * 1e-3) / 1e9
    traffic = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            tr = json.loads(tj.read_text())
            if tr.get("reads") == n and tr.get("docs") == D:
                traffic = tr.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(bank, reads, d_hits, args, D)

    line = {
        "metric": "k-mer x filter probes/s (150bp reads, ~100-species Bloom bank)",
        "value": value,
        "unit": "probes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded genomes + reads, no network)",
        "config": {
            "workload": "config2: 1M x 150bp reads/GPU vs D=100 COBS classic species bank",
            "reads_per_gpu": n, "read_len": args.read_len, "docs": D, "k": k, "num_hashes": h,
            "fpr": args.fpr, "sampling_step": args.step, "signature_rows": sig,
            "bank_device_bytes": int(info.device_bytes),
            "kmers_per_gpu": kmers_per_rank,
            "parallelism": f"reads sharded x{world}, bank replicated, RCCL all-reduce of D+1 totals",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "probe_cobs_kernel<21,7>", "probe_ms_avg": probe_ms,
            "probe_ms_max": probe_ms_max, "probe_launches": launches,
            "algo_bytes_per_launch": algo_bytes,
        },
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    bank.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(bank, reads, d_hits, args, D):
    """Oracle C restatement on a bounded sample of the same reads (rank 0, N=1)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # checker + CPU baseline only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    info = bank.info
    ob = oracle.CobsBank(bank.download(), [int(info.signature_rows)], int(info.page_size), D,
                         int(info.num_hashes), int(info.term_size))
    from xspect_amd.packing import pack_fixed

    def run(m):
        pr = pack_fixed(reads[:m])
        t = time.perf_counter()
        hits, nk = ob.query_packed(pr.buf, pr.offsets, step=args.step, threads=threads)
        return time.perf_counter() - t, hits, nk

    m = min(reads.shape[0], 20_000)
    dt, _, _ = run(m)
    m2 = int(min(reads.shape[0], max(m, m * args.cpu_seconds / max(dt, 1e-3))))
    dt, hits, nk = run(m2)
    gpu = d_hits[:m2].cpu().numpy().view(np.uint32)
    mism = int(np.count_nonzero(gpu != hits))
    probes = int(nk.sum()) * D
    return {
        "value": probes / dt, "unit": "probes/s", "cores": threads, "kind": "port",
        "sample": f"{m2} of the benchmark reads ({int(nk.sum())} k-mers x {D} docs) in {dt:.1f}s "
                  f"with the C oracle (OpenMP, {threads} threads)",
        "parity_sample_mismatches": mism,
    }


if __name__ == "__main__":
    main()
