"""Throughput of the k-mer x filter probe path on MI355X (driver contract).

    python bench.py [--gpus N --steps K --warmup W] [--workload species|genus|mlst|multigenus]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment (no torchrun around
it), bench.py starts the N ranks itself (launch_ranks: one child process per
GPU, started before anything touches the GPU) and prints rank 0's line; under
torchrun it is one of the ranks.  Either way the line carries the process
group's backend and size (dist_backend, rccl_world), every rank's GPU (PCI
address; two ranks on one device is an error outside the shared-GPU
rehearsal) and every rank's timed region and probe time (per_rank).

Default workload = BASELINE.json configs[1] / SURVEY.md §8(d) config 2: 1M
synthetic 150 bp reads per GPU against a D=100 species COBS classic bank
(k=21, h=7, fpr=0.01; 38.4M rows, 0.5 GB file / 0.61 GB in HBM, larger than
the 256 MiB Infinity Cache).  One step = one query of the whole read batch,
resident in HBM (units -> scan -> scatter -> probe -> totals).  With N>1
ranks the D+1 per-doc totals (the input of the SVM vector) are all-reduced
over RCCL: reads sharded (seed 42+rank), bank replicated, weak scaling; at
N > 1 each rank takes 12.5M reads by default, so N=8 is BASELINE.json
configs[2] (config 3: 100M reads over 8 GPUs) at its stated size.

Every rank checks its own values after the timed region (`checks`): its hit
rows of 3,000 reads against the C oracle, its local totals against its hit
matrix, and (rank 0) the all-reduced totals against the host sum of the
all-gathered per-rank totals; multigenus checks its exchanged column blocks
by checksums.  A failed check prints the line and exits with status 3.

Other workloads (SURVEY.md §8(d) configs 4/5 and the genus path):
  genus       rbloom filter over all 100 genomes (k=21, fpr=0.01), D=1
  mlst        7 loci x 1430 alleles, COBS compact (k=31, h=1, fpr=0.001,
              64-byte pages = 512 alleles per doc group); one step probes all loci
  multigenus  each rank holds a different 100-species bank, reads replicated;
              rank q ends with every bank's hit columns for its 1/N of the
              reads (one RCCL all-to-all; docs sharded, output by reads)

metric = k-mer x filter probes/s = sum(ceil((L-k+1)/step)) x docs / second,
whole job.  roofline prices the probe alone (HIP events on its launch
stream around every probe of the timed region) at its algorithmic bytes.
Species banks of 32 MiB and more take the partitioned COBS pipeline (bucket ->
per-XCD L2 lookup -> resolve), genus filters of 16 MiB and more on member-rich
input the partitioned rbloom pipeline: SURVEY.md §8(d)'s 64 B per row or
filter word (h or K per k-mer).  The direct kernels: one 128-byte L2 line fill per random row (COBS: h rows per
k-mer and doc group; rbloom: K dwords per k-mer; MLST: the 64-byte rows
themselves, its banks being Infinity-Cache resident).  Both + the read bytes,
hit matrix and per-read metadata; peak = 8.0 TB/s; traffic = PMC bytes per
probe from profiles/r06_traffic.json.  cpu_baseline: the C oracle (oracle/liboracle.so,
OpenMP) on a bounded sample of the same reads and bank (rank 0, N=1 only);
its hits are also compared with the GPU's; plus the reference's per-read loop
shape on one core.  host_path: the same step from host buffers (PCIe).
end_to_end (species/genus, N=1): SURVEY.md §8(d) time (ii), the same reads as
a FASTQ file -> totals / hit matrix through the library's file path.
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
# Infinity-Cache (MALL) ceiling for random row gathers: /opt/skills/guides/MI355X_MICROARCH.md
# "Indexed rows: gather into LDS", 38 MB table of uniformly random rows: 8.6 TB/s chip-wide
MALL_PEAK_GBS = 8600.0
# L2 request ceiling of one XCD's gathers from an L2-resident table, all 8 XCDs:
# 268 G requests/s whatever the size (4 or 16 B), depth or occupancy (profiles/r02_l2gather.txt)
L2_GATHER_PEAK_REQ = 268e9
# BASELINE.json "metric", verbatim (the line reports one N of the 1/2/4/8 curve)
METRIC = "k-mer\u00d7filter probes/s (150bp reads, ~100-species Bloom bank) at 1/2/4/8 GPUs"
# Bytes one random row (or filter dword) costs: the gfx950 L2 fills a whole
# 128-byte line per miss.  SURVEY.md §8(d) prices a row at 64 B "unless rocprof
# shows 128 B fills"; profiles/r01_pmc_probe.txt shows TCC_EA0_RDREQ_128B ==
# TCC_EA0_RDREQ (915.9 M per launch, 32B/64B requests ~0), so 128 B it is.
ROW_BYTES = 128
# SURVEY.md §8(d)'s per-row figure, used for the partitioned COBS pipeline,
# which reads rows from L2-resident bank partitions instead of random lines.
SURVEY_ROW_BYTES = 64
# Rehearsal of the N>1 path on a one-GPU box: every rank on cuda:0, gloo
# collectives through host copies (RCCL does not share a device between ranks).
SHARE_GPU = os.environ.get("XSPECT_BENCH_SHARE_GPU") == "1"
# BASELINE.json configs[2]: 100M reads sharded over 8 GPUs = 12.5M per GPU
CONFIG3_READS_PER_GPU = 12_500_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="species", choices=["species", "genus", "mlst", "multigenus"])
    ap.add_argument("--reads", type=int, default=None,
                    help="reads per GPU (default: 1M at --gpus 1 = config 2; species at --gpus N > 1: 12.5M, "
                         "so N=8 is config 3's 100M reads; other workloads 1M)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--docs", type=int, default=100)
    ap.add_argument("--genome-len", type=int, default=4_000_000)
    ap.add_argument("--step", type=int, default=1, help="sparse sampling step")
    ap.add_argument("--genus-filter-frac", type=float, default=1.0,
                    help="genus: build the filter from this fraction of the genomes (reads come from all)")
    ap.add_argument("--k", type=int, default=None, help="species/multigenus: k-mer length (default 21)")
    ap.add_argument("--hashes", type=int, default=7, help="species/multigenus: COBS num_hashes (default 7)")
    ap.add_argument("--mlst-foreign", type=float, default=0.0,
                    help="mlst: fraction of reads from outside every locus (WGS-like input: ~1.0)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check-reads", type=int, default=3000,
                    help="reads per rank whose GPU hit rows are compared with the C oracle (every N)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the PCIe-inclusive host-buffer runs (profiling: only full-size probe launches)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end legs (the bench's reads as a FASTQ file -> totals / hit matrix)")
    ap.add_argument("--totals-only", action="store_true",
                    help="diagnostic: probe without writing the per-read hit matrix (totals only)")
    ap.add_argument("--probe-path", default="auto", choices=["auto", "direct", "partitioned"],
                    help="diagnostic: the banks' probe path (xs_bank_set_probe_options; auto = the production "
                         "choice, direct = the gather kernels, partitioned = the partitioned probes forced)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "r06_traffic.json"))
    ap.add_argument("--rccl-world1", action="store_true",
                    help="rehearsal: a one-rank RCCL process group running every collective of the N>1 path "
                         "(the all-reduce of totals or the column exchange, the per-rank gathers and checks) "
                         "on a one-GPU box")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launched N>1 runs: seconds before the parent kills every rank")
    args = ap.parse_args()
    if args.reads is None:
        n_gpus = int(os.environ.get("WORLD_SIZE", args.gpus))
        args.reads = CONFIG3_READS_PER_GPU if (n_gpus > 1 and args.workload == "species") else 1_000_000
    return args


def free_port() -> int:
    """A TCP port on 127.0.0.1 that nothing listens on right now."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, cmd: list[str], timeout: float, env: dict | None = None, poll_s: float = 0.2) -> int:
    """One child process per rank (the reference's only fan-out is one process
    per input, scripts/benchmark/classify/main.nf:1-22; here one per GPU).

    Each child gets RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
    MASTER_ADDR=127.0.0.1 and a free MASTER_PORT, as torchrun would set them.
    The parent touches no GPU and never execs: it starts the children, copies
    rank 0's JSON line to its stdout (rank 0's other stdout lines go to
    stderr), lets every rank's stderr through, and waits.  If a child fails, or the whole run outlives
    `timeout`, the remaining children are killed and the parent returns
    non-zero (the first failing child's code, 124 on timeout)."""
    import subprocess
    import threading

    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(free_port()))
    procs = []
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    except BaseException:
        for p in procs:
            p.kill()
        raise

    def forward(stream):
        # the JSON line to stdout; anything else rank 0 prints there (gloo's
        # connection notes, for one) to stderr, so stdout stays one line
        for line in iter(stream.readline, b""):
            out = sys.stdout if line.lstrip().startswith(b"{") else sys.stderr
            out.buffer.write(line)
            out.flush()

    fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    fwd.start()
    deadline = time.monotonic() + timeout
    code = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            r, code = bad[0]
            print(f"bench launcher: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            print(f"bench launcher: ranks still running after {timeout:.0f}s; stopping them", file=sys.stderr,
                  flush=True)
            code = 124
            break
        time.sleep(poll_s)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    fwd.join(timeout=10)
    return code if code >= 0 else 128 - code  # a signal -s becomes 128 + s, as a shell reports it


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class Workload:
    """Banks + a step closure for one benchmark configuration."""

    def __init__(self, args, rank, world, dev, stream, pg=False):
        import torch
        from xspect2_amd.bank import Bank, bloom_parameters, cobs_signature_size
        from xspect2_amd.synth import make_genomes, make_reads

        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        self.pg = pg  # a process group: the N>1 collectives run (also at world 1 under --rccl-world1)
        s = stream.cuda_stream
        self.stream = s
        w = args.workload
        self.k = 31 if w == "mlst" else (args.k or 21)
        self.banks = []
        self.config = {}
        self.row_bytes = ROW_BYTES
        self.roofline_note = None
        if w in ("species", "genus", "multigenus"):
            gseed = 42 + (1000 * rank if w == "multigenus" else 0)
            genomes = make_genomes(args.docs, args.genome_len, seed=gseed)
            g_dev = torch.from_numpy(genomes.reshape(-1)).to(dev)
            g_offs = torch.arange(args.docs + 1, dtype=torch.int64, device=dev) * args.genome_len
            if w == "genus":
                nf = max(1, int(round(args.docs * args.genus_filter_frac)))
                n_items = genomes[:nf].size - self.k + 1  # Bloom(total_length - k + 1, fpr), :82-88
                nbytes, nh = bloom_parameters(n_items, 0.01)
                bank = Bank.create_bloom(self.k, nbytes, nh, device=dev.index)
                bank.build_device(g_dev, genomes[:nf].size, g_offs[:nf + 1], nf, None, stream=s)
                self.config.update(genomes_in_filter=nf)
                self.config.update(bloom_bytes=nbytes, bloom_hashes=nh)
                self.rows_per_kmer = nh
                self.kernel = f"probe_bloom_kernel<21,{nh},2> (2 bits first, the rest if both set)"
            else:
                h = args.hashes
                sig = cobs_signature_size(args.genome_len - self.k + 1, h, 0.01)
                bank = Bank.create_cobs(self.k, h, [sig], args.docs,
                                        [f"species_{gseed}_{i:03d}" for i in range(args.docs)],
                                        device=dev.index)
                g_docs = torch.arange(args.docs, dtype=torch.int32, device=dev)
                bank.build_device(g_dev, genomes.size, g_offs, args.docs, g_docs, stream=s)
                self.config.update(signature_rows=sig, num_hashes=h, fpr=0.01)
                self.rows_per_kmer = h
                # a row costs the 128-B lines its padded device pitch spans (two at D > 1024)
                self.row_bytes = max(ROW_BYTES, -(-bank.info.device_row_pitch // ROW_BYTES) * ROW_BYTES)
                nch = -(-args.docs // 128)  # 16-byte chunks of a row
                if (self.k, h) in ((21, 7), (31, 1)) and args.docs <= 128:
                    self.kernel = f"probe_cobs_fast<{self.k},{h}>"
                elif 2 <= nch <= 16:
                    lanes = 2 if nch == 2 else 4 if nch <= 4 else 8 if nch <= 8 else 16
                    self.kernel = f"probe_cobs_wide<k={self.k},h={h},C={lanes}> (D={args.docs})"
                else:
                    self.kernel = f"probe_cobs (k={self.k}, h={h}, D={args.docs})"
            torch.cuda.synchronize(dev)
            del g_dev
            log(rank, f"bank built ({bank.info.device_bytes / 1e9:.2f} GB); generating {args.reads} reads per rank")
            self.banks = [bank]
            rseed = 42 if w == "multigenus" else 42 + rank  # multigenus: same reads on every rank
            reads, _ = make_reads(genomes if w != "multigenus" else make_genomes(args.docs, args.genome_len, 42),
                                  args.reads, args.read_len, seed=rseed)
        else:  # mlst
            reads, loci_info = self._mlst(args, dev, s)
            self.config.update(loci=len(self.banks), **loci_info)
            self.kernel = "probe_cobs_vslice<31,3> (compact, 3 groups of 64-B pages; one lane per 32 docs, bit-sliced counters)"
        if args.probe_path != "auto":  # diagnostic runs of one path (the default line never sets it)
            mode = {"direct": 0, "partitioned": 2}[args.probe_path]
            for b in self.banks:
                b.set_probe_options(cobs_part=mode, bloom_part=mode)
            self.config.update(probe_path=args.probe_path)
        self.reads = reads
        self.n = reads.shape[0]
        self.seq_bytes = reads.size
        self.d_seqs = torch.from_numpy(reads.reshape(-1)).to(dev)
        self.d_offs = torch.arange(self.n + 1, dtype=torch.int64, device=dev) * args.read_len
        self.docs = [b.num_docs for b in self.banks]
        self.d_hits = [torch.empty((self.n, d), dtype=torch.int32, device=dev) for d in self.docs]
        self.d_nk = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.d_tot = [torch.zeros(d + 1, dtype=torch.int64, device=dev) for d in self.docs]
        self.nk_read = (args.read_len - self.k + args.step) // args.step
        self.kmers = self.n * self.nk_read
        if w == "multigenus" and pg:
            # the library's docs-sharded gather (xspect2_amd.distributed): hit rows
            # travel in the narrowest type that holds a read's k-mer count (1 byte
            # for 150 bp reads), narrowed and widened on the device; the layout
            # (docs per rank, wire type) is agreed once, as a serving loop would
            from xspect2_amd.distributed import doc_shard_layout
            from xspect2_amd.distributed import shard_range
            self.layout = doc_shard_layout(self.docs[0], self.nk_read)
            self.counts = [b - a for a, b in (shard_range(self.n, q, world) for q in range(world))]
            self.config["exchange_dtype"] = str(self.layout[1]).replace("torch.", "")
            self.config["exchanged_docs"] = sum(self.layout[0])
            self.config["reads_out_per_rank"] = self.counts

    def _mlst(self, args, dev, s):
        import torch
        from xspect2_amd.bank import Bank, cobs_signature_size
        rng = np.random.default_rng(4242)
        acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
        loci, n_alleles, page = 7, 1430, 64
        all_alleles = []
        group_rows = []
        for li in range(loci):
            base = acgt[rng.integers(0, 4, 620)]
            alleles = []
            for _ in range(n_alleles):
                L = int(rng.integers(400, 601))
                a = base[:L].copy()
                pos = rng.integers(0, L, int(rng.integers(0, 12)))
                a[pos] = acgt[(np.searchsorted(acgt, a[pos]) + 1) % 4]
                alleles.append(a)
            order = sorted(range(n_alleles), key=lambda i: (alleles[i].size, i))
            alleles = [alleles[i] for i in order]
            all_alleles.append(alleles)
            per = 8 * page
            sig = [cobs_signature_size(max(a.size for a in alleles[g:g + per]) - self.k + 1, 1, 0.001)
                   for g in range(0, n_alleles, per)]
            group_rows.append(sig)
            bank = Bank.create_cobs(self.k, 1, sig, n_alleles, [f"Allele_ID_{i}" for i in range(n_alleles)],
                                    page_size=page, compact=True, device=dev.index)
            buf = np.concatenate(alleles)
            offs = np.zeros(n_alleles + 1, dtype=np.int64)
            offs[1:] = np.cumsum([a.size for a in alleles])
            bank.build_device(torch.from_numpy(buf).to(dev), buf.size, torch.from_numpy(offs).to(dev),
                              n_alleles, torch.arange(n_alleles, dtype=torch.int32, device=dev), stream=s)
            self.banks.append(bank)
        torch.cuda.synchronize(dev)
        # reads: 150 bp windows of random alleles of random loci, 1 % errors
        n = args.reads
        li = rng.integers(0, loci, n)
        ai = rng.integers(0, n_alleles, n)
        reads = np.empty((n, args.read_len), dtype=np.uint8)
        for i in range(n):
            a = all_alleles[li[i]][ai[i]]
            st = int(rng.integers(0, a.size - args.read_len + 1))
            reads[i] = a[st:st + args.read_len]
        if args.mlst_foreign > 0:  # reads from elsewhere in the genome: random sequence
            nf = int(round(args.mlst_foreign * n))
            reads[:nf] = acgt[rng.integers(0, 4, (nf, args.read_len))]
        self.rows_per_kmer = sum(len(g) for g in group_rows)  # one 64-B row per group per locus
        # a locus bank (~97 MB) stays in the 256 MB Infinity Cache: count the
        # row itself (page bytes), not an HBM line fill
        self.row_bytes = page
        self.roofline_note = ("bound = mall: locus banks (~97 MB each) are Infinity-Cache resident, rows arrive "
                              "as 128-B line fills from the MALL (or hit L2), not HBM; achieved counts the 64-B rows "
                              "themselves; peak = the guide's random-row gather rate from a 38 MB (Infinity-Cache) "
                              "table, 8.6 TB/s")
        return reads, {"alleles_per_locus": n_alleles, "page_size": page, "k": self.k,
                       "foreign_read_frac": args.mlst_foreign,
                       "num_hashes": 1, "fpr": 0.001,
                       "signature_rows": int(sum(sum(g) for g in group_rows))}

    def step(self):
        for b, h, t in zip(self.banks, self.d_hits, self.d_tot):
            b.query_device(self.d_seqs, self.seq_bytes, self.d_offs, self.n, self.args.step,
                           None if self.args.totals_only else h, self.d_nk, t, stream=self.stream)
        if self.pg:
            from xspect2_amd import distributed
            if self.args.workload == "multigenus":
                # docs sharded, output sharded by reads: every rank's hit columns of
                # rank q's 1/N of the reads go to rank q over xGMI (one all-to-all in
                # the narrowest exact type) -> [n/N, sum D_r] per rank
                self.exchanged = distributed.exchange_doc_columns(self.d_hits[0], self.counts, *self.layout)
            else:
                for t in self.d_tot:
                    distributed.allreduce_(t)  # per-doc totals + k-mer total over all ranks

    def probes_per_step(self):
        per_rank = self.kmers * sum(self.docs)
        return per_rank * self.world

    def algo_bytes_per_launch(self):
        """Bytes one probe launch must move (per bank; averaged over banks)."""
        if getattr(self, "partitioned", False):
            # SURVEY.md §8(d)'s algorithmic figure for both partitioned pipelines:
            # one random 64-B transaction per row (COBS: h per k-mer) or filter
            # word (rbloom: K per k-mer), + the read bytes, hit rows and per-read
            # metadata.  The pipelines fetch no row or word as a random HBM line
            # (their PMC traffic per step is below this figure).
            d = self.docs[0]
            return (self.kmers * self.rows_per_kmer * SURVEY_ROW_BYTES + self.seq_bytes + self.n * d * 4
                    + self.n * (8 + 4 + 8 + 8))
        per_bank = []
        for d in self.docs:
            rows = self.rows_per_kmer if self.args.workload != "mlst" else self.rows_per_kmer / len(self.docs)
            # rows + the read bytes (one window pass) + hit rows + per-read metadata
            per_bank.append(self.kmers * rows * self.row_bytes + self.seq_bytes + self.n * d * 4
                            + self.n * (8 + 4 + 8 + 8))
        return sum(per_bank) / len(per_bank)


def build_id() -> str:
    """The loaded library's build id (a hash of its sources, xspect2_amd/build.py)."""
    from xspect2_amd import _lib
    return _lib.build_id()


def check_distinct_devices(dev) -> list[str]:
    """PCI address of every rank's GPU (all-gathered); raises if two ranks
    drive the same device, which would make an N-GPU line an N-rank-on-one-GPU
    line.  Skipped (addresses still returned) in the shared-GPU rehearsal."""
    import torch
    import torch.distributed as dist
    p = torch.cuda.get_device_properties(dev)
    mine = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    addrs: list = [None] * dist.get_world_size()
    dist.all_gather_object(addrs, mine)
    if not SHARE_GPU and len(set(addrs)) != len(addrs):
        raise RuntimeError(f"ranks share a GPU (PCI addresses by rank: {addrs}); one rank per GPU is required")
    return addrs


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start one process per GPU ourselves, before
        # anything here touches the GPU (torch.cuda is not imported yet)
        sys.exit(launch_ranks(args.gpus, [sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]],
                              args.launch_timeout))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if SHARE_GPU:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_info = {"dist_backend": None, "rccl_world": None, "rank_devices": None}
    pg = world > 1 or args.rccl_world1
    if pg:
        if world == 1:  # --rccl-world1
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if SHARE_GPU:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        dist_info = {"dist_backend": dist.get_backend(), "rccl_world": dist.get_world_size(),
                     "rank_devices": check_distinct_devices(dev)}
        if dist_info["rccl_world"] != world:
            raise RuntimeError(f"process group has {dist_info['rccl_world']} ranks, WORLD_SIZE={world}")
    stream = torch.cuda.current_stream(dev)
    t_setup = time.time()
    wl = Workload(args, rank, world, dev, stream, pg)
    log(rank, f"{args.workload}: {len(wl.banks)} bank(s), docs={wl.docs}, "
              f"{sum(b.info.device_bytes for b in wl.banks) / 1e9:.2f} GB in HBM, setup {time.time() - t_setup:.1f}s")

    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize(dev)
    for b in wl.banks:
        b.set_profiling(True)
        b.probe_stats()  # reset
        b.probe_rows()
        b.pass_stats()
    if pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    torch.cuda.synchronize(dev)
    if pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    launches, probe_ms_total, probe_ms_max = 0, 0.0, 0.0
    rows_read = 0
    passes = {}
    for b in wl.banks:
        rows_read += b.probe_rows()
        for name, (ms, cnt) in b.pass_stats().items():
            t, c = passes.get(name, (0.0, 0))
            passes[name] = (t + ms, c + cnt)
        b.set_profiling(False)
        n_l, tot_ms, mx = b.probe_stats()
        launches += n_l
        probe_ms_total += tot_ms
        probe_ms_max = max(probe_ms_max, mx)
    probe_ms = probe_ms_total / max(1, launches)
    per_rank = None
    if pg:
        # every rank's own timed region and probe time; the line's time is the max
        parts = all_gather_host(torch.tensor([elapsed, probe_ms], dtype=torch.float64), world)
        el = [float(p[0].item()) for p in parts]
        pm = [float(p[1].item()) for p in parts]
        elapsed = max(el)
        per_rank = {"elapsed_s": el, "probe_ms_avg": pm, "probe_ms_min": min(pm), "probe_ms_max": max(pm)}

    # sanity of the last step: whole-job k-mer totals
    for t in wl.d_tot:
        tot = t.cpu().numpy().view(np.uint64)
        want = wl.kmers * (world if args.workload != "multigenus" else 1)
        assert int(tot[-1]) == want, f"k-mer total {int(tot[-1])} != {want}"
    if args.workload == "genus":  # member k-mers / sampled k-mers (steers the rbloom probe path)
        wl.config["member_fraction"] = round(int(tot[0]) / max(1, int(tot[-1])), 4)
    # every rank checks its own values (oracle sample, totals, exchanged columns); outside the timed region
    checks = self_check(wl, args, rank, world, dev, pg)

    value = wl.probes_per_step() * args.steps / elapsed
    from xspect2_amd._lib import XS_PATH_PARTITIONED
    wl.partitioned = args.workload == "genus" and wl.banks[0].probe_path() == XS_PATH_PARTITIONED
    if args.workload in ("species", "multigenus") and wl.banks[0].probe_path() == XS_PATH_PARTITIONED:
        wl.partitioned = "cobs"
        wl.kernel = (f"COBS partitioned: cobs_bucket<{wl.k},{wl.rows_per_kmer},2048> (hash, bin rows by 2 MiB bank "
                     "partition) -> cobs_lookup (per-XCD L2-resident partition, rows back in entry order) -> "
                     "cobs_resolve (AND per k-mer in LDS, per-read counts)")
        wl.row_bytes = SURVEY_ROW_BYTES
        wl.roofline_note = ("achieved = SURVEY.md §8(d)'s algorithmic bytes (h x 64 B per k-mer + reads, hits, "
                            "metadata) over the whole probe (HIP events around the pipeline); traffic = PMC HBM "
                            "bytes of the pipeline per step, below the algorithmic figure: rows come from "
                            "L2-resident partitions, not random HBM lines.  Per-kernel bounds: bucket = VALU issue "
                            "(XXH64 x h + Barrett), lookup = vector-L1 miss path to L2 (TCP pending "
                            "stalls), resolve = HBM streaming; see DESIGN.md")
    elif wl.partitioned:
        wl.kernel = ("rbloom partitioned: bloom_bucket (hash, bin by 2 MiB filter partition) -> "
                     "bloom_lookup (per-XCD L2-resident partition) -> resolve -> count")
        wl.row_bytes = SURVEY_ROW_BYTES
        wl.roofline_note = ("achieved = SURVEY.md §8(d)'s algorithmic bytes (K x 64 B per k-mer + reads, hits, "
                            "metadata) over the whole probe (HIP events around the pipeline); traffic = PMC HBM "
                            "bytes of the pipeline per step, below the algorithmic figure.  Per-kernel bounds: "
                            "bucket = VALU (XXH3, LCG, Barrett), lookup = vector-L1 miss path to L2; see DESIGN.md")
    elif rows_read:  # rbloom: the data-dependent count of filter words loaded
        wl.rows_per_kmer = rows_read / max(1, launches) / wl.kmers
    algo_bytes = wl.algo_bytes_per_launch()
    achieved = algo_bytes / (probe_ms * 1e-3) / 1e9
    # MLST locus banks (~97 MB) are Infinity-Cache resident
    peak = MALL_PEAK_GBS if args.workload == "mlst" else HBM_PEAK_GBS
    traffic = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            data = json.loads(tj.read_text())
            # multigenus runs the species kernel on a bank of the same size
            tr = data.get(args.workload) or (data.get("species") if args.workload == "multigenus" else None) or {}
            if tr.get("reads") == wl.n:  # measured on this workload at this size
                traffic = tr.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if wl.partitioned:  # the whole partitioned pipeline per query (profiles/r06_traffic.json, from r06_pmc_cobspart.json and r06_pmc_bloompart.json)
        traffic = None
        try:
            key = "species_partitioned" if wl.partitioned == "cobs" else "genus_partitioned"
            tp = json.loads(tj.read_text()).get(key) or {}
            if tp.get("reads") == wl.n:
                traffic = tp.get("hbm_bytes_per_step")
        except Exception:
            traffic = None
    pass_ms = {name: ms / max(1, launches) for name, (ms, cnt) in passes.items() if cnt}
    lookup_l2 = None
    if wl.partitioned and "lookup" in pass_ms:
        # the dominant pass against its own ceiling: L2 requests per launch (PMC,
        # scaled to this call's k-mers) over the lookup's live HIP-event time
        pmc_file, prefix = (("r06_pmc_cobspart.json", "xs::cobs_lookup_kernel") if wl.partitioned == "cobs" else
                            ("r06_pmc_bloompart.json", "xs::bloom_lookup_kernel"))
        try:
            pmc = json.loads((ROOT / "profiles" / pmc_file).read_text())["kernels"]
            key = next(k for k in pmc if k.startswith(prefix))
            req = pmc[key]["TCC_REQ_sum"] * wl.kmers / (1_000_000 * 130)
            ach = req / (pass_ms["lookup"] * 1e-3)
            lookup_l2 = {"kernel": key, "bound": "l2_requests", "achieved": ach, "peak": L2_GATHER_PEAK_REQ,
                         "unit": "req/s", "frac": ach / L2_GATHER_PEAK_REQ, "requests_per_launch": req,
                         "lookup_ms_avg": pass_ms["lookup"],
                         "l2_hit_rate": pmc[key].get("l2_hit_rate"),
                         "source": f"TCC_REQ_sum per dispatch from profiles/{pmc_file} (1 M reads; "
                                   "scaled by k-mers); peak = pure L2 gathers, profiles/r02_l2gather.txt"}
        except Exception:
            lookup_l2 = None
    if world > 1:
        # the PMC files are one-GPU, 1M-read measurements: they describe no rank of this run
        traffic, lookup_l2 = None, None
    # the PCIe-inclusive legs are a per-GPU figure: measured at N=1 only
    host = None if args.no_host_path or world > 1 else host_path(wl, args)
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and args.workload in ("species", "genus"):
        e2e = end_to_end(wl, args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, args)

    nr = f"{wl.n / 1e6:g}M x {args.read_len}bp reads"
    if world > 1 and wl.n == CONFIG3_READS_PER_GPU:
        species_cfg = (f"config3: {wl.n * world / 1e6:g}M x {args.read_len}bp reads sharded over {world} GPUs "
                       f"({nr}/GPU; N=8 = BASELINE configs[2]'s 100M)")
    elif world > 1:
        species_cfg = f"species: {nr}/GPU sharded over {world} GPUs (config 3's layout, not its size)"
    else:
        species_cfg = ("config3 per-GPU shard (100M reads / 8 GPUs)" if wl.n == CONFIG3_READS_PER_GPU else
                       "config2" if wl.n == 1_000_000 else "species") + f": {nr}/GPU"
    names = {"species": f"{species_cfg} vs D={args.docs} COBS classic species bank",
             "genus": f"genus path: {nr}/GPU vs rbloom filter over {args.docs} genomes",
             "mlst": f"config4: {nr}/GPU vs 7 loci x 1430 alleles (COBS compact)",
             "multigenus": f"config5: {nr} vs one {args.docs}-species bank per GPU, hit columns exchanged to the reads' ranks"}
    par = {"species": f"reads sharded x{world}, bank replicated, RCCL all-reduce of D+1 totals",
           "genus": f"reads sharded x{world}, filter replicated, RCCL all-reduce of totals",
           "mlst": f"reads sharded x{world}, loci banks replicated, RCCL all-reduce of totals",
           "multigenus": f"docs sharded x{world} (one bank per GPU), reads replicated, output sharded by reads: RCCL "
                         "all-to-all of hit columns in the narrowest exact integer type"}
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "probes/s",
        "n_gpus": world,
        **dist_info,
        "per_rank": per_rank,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "build_id": build_id(),
        "data": "synthetic (seeded genomes + reads, no network)",
        "config": {
            "workload": names[args.workload],
            "reads_per_gpu": wl.n, "read_len": args.read_len, "docs_per_bank": wl.docs[0],
            "banks": len(wl.banks), "k": wl.k, "sampling_step": args.step,
            "bank_device_bytes": int(sum(b.info.device_bytes for b in wl.banks)),
            "kmers_per_gpu": wl.kmers, "parallelism": par[args.workload], **wl.config,
        },
        "roofline": {
            "bound": "mall" if args.workload == "mlst" else "hbm", "achieved": achieved, "peak": peak,
            "unit": "GB/s", "frac": achieved / peak, "traffic": traffic,
            "traffic_frac": (traffic / (probe_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
            **({"traffic_note": "traffic, traffic_frac and lookup_l2 are one-GPU PMC figures (profiles/): "
                                "not reported at N > 1"} if world > 1 else {}),
            "frac_basis": ("frac = SURVEY.md §8(d)-priced algorithmic bytes / probe time / peak; traffic_frac = "
                           "PMC-measured HBM bytes of the same probe (traffic) / probe time / 8 TB/s: the bytes "
                           "the pipeline really moves, intermediates included" if traffic else
                           "frac = algorithmic bytes / probe time / peak"),
            "kernel": wl.kernel,
            "probe_ms_avg": probe_ms, "probe_ms_max": probe_ms_max, "probe_launches": launches,
            "pass_ms_avg": pass_ms or None, "lookup_l2": lookup_l2,
            "algo_bytes_per_launch": algo_bytes, "row_bytes": wl.row_bytes, "rows_per_kmer": wl.rows_per_kmer,
            **({"note": wl.roofline_note} if wl.roofline_note else {}),
        },
        "cpu_baseline": cpu,
        "checks": checks,
        "host_path": host,
        "end_to_end": e2e,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    for b in wl.banks:
        b.close()
    if pg:
        dist.destroy_process_group()
    if not checks["ok"]:
        sys.exit(3)


def oracle_banks(wl):
    """The C oracle over copies of this rank's banks (checker + CPU baseline only)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    if getattr(wl, "_obanks", None) is None:
        wl._obanks = []
        for b in wl.banks:
            inf = b.info
            if inf.kind == 2:
                wl._obanks.append(oracle.BloomFilter(b.download(), int(inf.num_hashes), int(inf.term_size)))
            else:
                wl._obanks.append(oracle.CobsBank(b.download(), b.signature_sizes(), int(inf.page_size),
                                                  int(inf.num_docs), int(inf.num_hashes), int(inf.term_size)))
    return wl._obanks


def all_gather_host(t, world: int) -> list:
    """Every rank's copy of tensor `t`, in rank order, on the host: the
    collective runs on the current GPU under RCCL (nccl wants device tensors
    for input and outputs alike) and on the CPU under gloo."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    src = t.to(dev)
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src)
    return [p.cpu() for p in parts]


def _checksum(x, row0: int):
    """Position-weighted int64 checksum of an integer matrix block whose first
    row is row `row0` of its job-wide matrix (equal blocks <=> equal sums, up to
    collisions ~2^-63): sum of value * (global row * 1000003 + col + 1)."""
    import torch
    n, d = x.shape
    r = torch.arange(row0, row0 + n, dtype=torch.int64, device=x.device)[:, None]
    c = torch.arange(d, dtype=torch.int64, device=x.device)[None, :]
    return int((x.to(torch.int64) * (r * 1000003 + c + 1)).sum().item())


def self_check(wl, args, rank, world, dev, pg=None):
    """Every rank checks the values of its last step (outside the timed region):

    * its GPU hit rows of `--check-reads` reads spread over its shard against
      the C oracle on a copy of its bank (mismatching (read, doc) cells);
    * read-sharded workloads: its local D+1 totals (one more query, no
      collective) against the column sums of its hit matrix and its k-mer
      counts; then rank 0 compares the all-reduced totals of the timed steps
      with the host sum of every rank's all-gathered local totals
      (result.py:76-90: the job totals the all-reduce must reproduce);
    * multigenus at N > 1: the exchanged columns against the rows each rank
      sent, by position-weighted checksums of every (bank rank, read rank)
      block, all-gathered (a checksum of checksums).
    Returns rank 0's view: every rank's counts, and `ok`."""
    import torch
    import torch.distributed as dist
    from xspect2_amd.packing import pack_fixed

    m = min(wl.n, max(0, args.check_reads))
    idx = np.unique(np.linspace(0, wl.n - 1, m).astype(np.int64)) if m else np.zeros(0, np.int64)

    def oracle_sample():
        mism, cells = 0, 0
        if idx.size:
            pr = pack_fixed(wl.reads[idx])
            for ob, d_h in zip(oracle_banks(wl), wl.d_hits):
                hits, _ = ob.query_packed(pr.buf, pr.offsets, step=args.step, threads=host_cpus()["share"])
                gpu = d_h[torch.from_numpy(idx).to(d_h.device)].cpu().numpy().view(np.uint32)
                mism += int(np.count_nonzero(gpu != hits.reshape(gpu.shape)))
                cells += gpu.size
        return {"oracle_sample_reads": int(idx.size), "oracle_sample_cells": cells, "oracle_mismatches": mism}

    mine = {}
    if args.workload != "multigenus":
        # local totals of one more query against the local hit matrix
        bad_local = 0
        local = []
        for b, h, t in zip(wl.banks, wl.d_hits, wl.d_tot):
            lt = torch.zeros_like(t)
            b.query_device(wl.d_seqs, wl.seq_bytes, wl.d_offs, wl.n, args.step, h, wl.d_nk, lt,
                           stream=wl.stream)
            torch.cuda.synchronize(dev)
            want = torch.cat([h.sum(0, dtype=torch.int64), wl.d_nk.sum().reshape(1)])
            bad_local += int((lt != want).sum().item())
            local.append(lt)
        mine.update(oracle_sample())  # the hit rows this query wrote (also under --totals-only)
        mine["local_totals_mismatches"] = bad_local
        loc = torch.cat(local).cpu()
        if pg:
            parts = all_gather_host(loc, world)
            host_sum = np.sum([p.numpy().view(np.uint64) for p in parts], axis=0, dtype=np.uint64)
        else:
            host_sum = loc.numpy().view(np.uint64)
        reduced = torch.cat([t.cpu() for t in wl.d_tot]).numpy().view(np.uint64)
        mine["allreduce_vs_host_sum_mismatches"] = int(np.count_nonzero(reduced != host_sum))
    else:
        mine.update(oracle_sample())
    if args.workload == "multigenus" and pg:
        from xspect2_amd.distributed import shard_range
        sent = torch.tensor([_checksum(wl.d_hits[0][a:b], a) for a, b in
                             (shard_range(wl.n, q, world) for q in range(world))], dtype=torch.int64)
        got = all_gather_host(sent, world)
        a, _ = shard_range(wl.n, rank, world)
        bad, c0 = 0, 0
        for r, d in enumerate(wl.layout[0]):
            bad += int(_checksum(wl.exchanged[:, c0:c0 + d], a) != int(got[r][rank].item()))
            c0 += d
        mine["exchange_block_mismatches"] = bad
    keys = sorted(k for k in mine if k.endswith("mismatches"))
    if pg:
        allm: list = [None] * world
        dist.all_gather_object(allm, mine)
    else:
        allm = [mine]
    out = {"per_rank": allm, "ok": all(r[k] == 0 for r in allm for k in keys)}
    if rank == 0 and not out["ok"]:
        print(f"bench self-check FAILED: {allm}", file=sys.stderr, flush=True)
    return out


def cpu_baseline(wl, args):
    """Oracle C restatement on a bounded sample of the same reads (rank 0, N=1)."""
    from xspect2_amd.packing import pack_fixed

    cpus = host_cpus()
    threads = cpus["share"]
    obanks = oracle_banks(wl)

    def run(m):
        pr = pack_fixed(wl.reads[:m])
        t = time.perf_counter()
        # the batched restatements (a tuned port: COBS rows / rbloom bit bytes prefetched across a
        # read's k-mers, Barrett remainders; COBS: seed-independent XXH64 terms once per k-mer, 4 docs
        # per add), the same hits as the scalar oracle bit for bit (tests/test_oracle.py)
        outs = [getattr(ob, "query_packed_batched", ob.query_packed)(pr.buf, pr.offsets, step=args.step,
                                                                     threads=threads) for ob in obanks]
        return time.perf_counter() - t, outs

    m = min(wl.n, 20_000)
    dt, _ = run(m)
    m2 = int(min(wl.n, max(m, m * args.cpu_seconds / max(dt, 1e-3))))
    dt, outs = run(m2)
    # The whole read set can take less than the target on many cores: repeat
    # passes over it so the timed sample is ~cpu_seconds of CPU work.
    passes = 1
    if dt < 0.5 * args.cpu_seconds:
        extra = max(1, int(args.cpu_seconds / max(dt, 1e-3)) - 1)
        dt += sum(run(m2)[0] for _ in range(extra))
        passes += extra
    ref_style = reference_style_baseline(wl, args, obanks)
    mism = 0
    probes = 0
    for (hits, nk), d_h in zip(outs, wl.d_hits):
        gpu = d_h[:m2].cpu().numpy().view(np.uint32)
        mism += int(np.count_nonzero(gpu != hits.reshape(gpu.shape)))
        probes += int(nk.sum()) * gpu.shape[1] * passes
    port = ("batched: prefetched rows, hoisted hash terms, 4 docs per add; equal to the scalar oracle"
            if type(obanks[0]).__name__ == "CobsBank" else
            "batched: a read's bit indices first (Barrett remainders), bytes prefetched ahead; "
            "equal to the scalar oracle")
    return {
        "value": probes / dt, "unit": "probes/s", "cores": threads, "kind": "port", "host_cpus": cpus,
        "sample": f"{passes} pass(es) over {m2} of the benchmark reads x {len(obanks)} bank(s) "
                  f"({probes} probes) in {dt:.1f}s with the C restatement ({port}; OpenMP, {threads} threads = every CPU "
                  f"this process may run on: affinity {cpus['affinity']}, cgroup quota {cpus['cgroup_quota']}; "
                  f"os.cpu_count() {cpus['os_cpu_count']})",
        "parity_sample_mismatches": mism,
        "reference_style": ref_style,
    }


def host_cpus() -> dict:
    """The host CPUs this process can use: os.cpu_count() (the machine),
    sched_getaffinity (nproc) and the cgroup v2 CPU quota (cpu.max), whose
    minimum is the share the CPU baseline runs on."""
    import math
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = total
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except Exception:
        quota = None
    share = min(aff, max(1, math.floor(quota))) if quota else aff
    return {"os_cpu_count": total, "affinity": aff, "cgroup_quota": quota, "share": share}


def host_path(wl, args, reps=3):
    """The same step from host buffers (SURVEY.md §8(d) time (i)): packed reads
    in pageable host memory -> H2D -> kernels -> D2H of the n x D hit matrix
    (xs_query), and of the totals only (xs_query_totals).  PCIe-inclusive;
    never the headline value, which starts with the reads in HBM."""
    from xspect2_amd.bank import max_kmers, narrowest_count_dtype, pinned_empty
    from xspect2_amd.packing import pack_fixed

    pr = pack_fixed(wl.reads)
    out = {}
    # hit matrix in the narrowest exact type (narrowed on the device), into a
    # pinned output reused call after call, as a serving loop holds it
    hdt = narrowest_count_dtype(max_kmers(pr, wl.k, args.step))
    outs = {id(b): pinned_empty((pr.n, b.num_docs), hdt) for b in wl.banks}
    def fresh(b):  # a never-touched pageable array: the OS faults each page as the copy-out reaches it
        return b.query(pr, step=args.step, out=np.empty((pr.n, b.num_docs), np.uint32))

    def touch(b):  # first-touch cost alone: one write per 4 KiB page of a fresh matrix-sized array
        np.empty((pr.n, b.num_docs), np.uint32).reshape(-1).view(np.uint8)[::4096] = 0

    for name, fn in (("hits", lambda b: b.query(pr, step=args.step, hit_dtype=hdt, out=outs[id(b)])),
                     ("hits_u32_pageable", lambda b: b.query(pr, step=args.step)),
                     ("hits_u32_fresh_pageable", fresh), ("first_touch_u32_matrix", touch),
                     ("totals", lambda b: b.query_totals(pr, step=args.step))):
        for b in wl.banks:  # warm
            fn(b)
        dt, release = 0.0, 0.0
        for _ in range(reps):
            for b in wl.banks:
                t = time.perf_counter()
                res = fn(b)
                t1 = time.perf_counter()
                del res  # the caller dropping its result: timed apart (a fresh array's unmap)
                dt += t1 - t
                release += time.perf_counter() - t1
        dt, release = dt / reps, release / reps
        out[name] = {"ms_per_step": dt * 1e3}
        if not name.startswith("first_touch"):
            out[name]["probes_per_s"] = wl.probes_per_step() / wl.world / dt
        if name == "hits_u32_fresh_pageable":
            out[name]["release_ms_per_step"] = release * 1e3
    out["hit_dtype"] = np.dtype(hdt).name
    out["note"] = ("per GPU, reads from pageable host memory: H2D + probe + D2H.  hits: the n x D matrix in "
                   f"{np.dtype(hdt).name} (narrowed on the device; counts <= k-mers per read) into a reused pinned "
                   "buffer (xs_query_hits); hits_u32_pageable: Bank.query's default, xs_query's uint32 matrix into "
                   "a pageable array from the recycled host pool (bank._HostPool: pages faulted once), the rows "
                   "crossing PCIe as uint8 and widened on the host behind the probe; hits_u32_fresh_pageable: the "
                   "same into a never-touched np.empty array allocated inside the time, which adds the OS's "
                   "first-touch faults (taken as 2 MiB pages by the copy-out's 8 threads), the array's release "
                   "(the OS unmapping it when the caller drops it) timed apart as release_ms_per_step; "
                   "first_touch_u32_matrix: allocate, one write per 4 KiB page from one thread and release, no "
                   "probe; totals: D+1 counters.  The headline value starts with the reads in HBM")
    return out


def end_to_end(wl, args, reps=3):
    """SURVEY.md §8(d) time (ii), end to end from a file: the bench's reads
    written as a FASTQ (ids r<i>, quality 'I'), then file -> per-doc totals
    and file -> hit matrix (narrowest exact type) through the library's file
    path (file_io.read_batches + Bank.query_totals / Bank.query, as
    predict_columnar streams a file), with the native reader in device mode
    (text to HBM, records found on the GPU; the models' default) and in host
    mode.  The file is in the page cache (just written): disk time is not in
    it.  Best of `reps` passes; never the headline value."""
    import shutil
    import tempfile
    from xspect2_amd.file_io import read_batches

    tmp = Path(tempfile.mkdtemp(prefix="xs_bench_e2e_"))
    try:
        fq = tmp / "reads.fastq"
        qual = b"I" * args.read_len
        with open(fq, "wb") as fh:
            for lo in range(0, wl.n, 100_000):
                fh.write(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, wl.reads[i].tobytes(), qual)
                                  for i in range(lo, min(wl.n, lo + 100_000))))
        size = fq.stat().st_size
        out = {"file_bytes": size, "reads": wl.n}
        for mode, dev in (("device_reader", wl.dev.index), ("host_reader", None)):
            for name, fn in (("totals", lambda b, pb: b.query_totals(pb, step=args.step)),
                             ("hits", lambda b, pb: b.query(pb, step=args.step, hit_dtype="auto"))):
                ts = []
                for _ in range(reps):
                    t = time.perf_counter()
                    n = 0
                    for batch in read_batches(fq, device=dev):
                        for b in wl.banks:
                            fn(b, batch if dev is not None else batch.packed)
                        n += batch.n
                    ts.append(time.perf_counter() - t)
                assert n == wl.n
                dt = min(ts)
                out[f"{mode}_{name}"] = {"ms": dt * 1e3, "first_ms": ts[0] * 1e3,
                                         "probes_per_s": wl.probes_per_step() / wl.world / dt,
                                         "file_GBps": size / dt / 1e9}
        out["note"] = ("file (page cache) -> parse -> probe -> totals (D+1 counters) or the n x D hit matrix in the "
                       "narrowest exact type, on host; device_reader: xs_fastx_open_device (the models' default "
                       "for file inputs), host_reader: xs_fastx_open + H2D of packed batches")
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def reference_style_baseline(wl, args, obanks, m=10_000):
    """SURVEY.md §8(d) CPU baseline (ii): the reference's loop shape, one
    native query per read from a Python loop plus the per-read result
    dictionary (probabilistic_filter_model.py:291-310, :227, :393-409), on one
    core over a 10k-read subset; extrapolated to probes/s."""
    import numpy as np

    m = min(m, wl.n)
    names = [[str(d) for d in range(n)] for n in wl.docs]
    t = time.perf_counter()
    probes = 0
    for i in range(m):
        read = wl.reads[i]
        buf = np.concatenate([read, np.zeros(1, dtype=np.uint8)])
        offs = np.array([0, read.size], dtype=np.uint64)
        for ob, nm in zip(obanks, names):
            hits, nk = ob.query_packed(buf, offs, step=args.step, threads=1)
            row = hits.reshape(-1)
            order = np.argsort(-row.astype(np.int64), kind="stable")
            _ = {nm[j]: int(row[j]) for j in order.tolist()}
            probes += int(nk[0]) * len(nm)
    dt = time.perf_counter() - t
    return {"value": probes / dt, "unit": "probes/s", "cores": 1,
            "sample": f"{m} reads, one oracle query + result dict per read from a Python loop, "
                      f"{dt:.1f}s (the reference's per-read loop shape; its C++/Rust libraries are absent)"}


if __name__ == "__main__":
    main()
