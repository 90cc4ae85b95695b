"""A/B of the partitioned COBS lookup's L2 prefetch (round 6, VERDICT r5 item
1), GPU.  Config-2 bank (D=100, built on the device), the bench's 1 M reads in
HBM.  For each call size (the reader windows of a 1 M-read file: 54 k, 107 k,
214 k, 429 k, 196 k reads, and one 1 M call) and each prefetch lead (rounds
of groups ahead; 0 = off), the probe's HIP-event time and the per-pass times
(xs_bank_pass_stats), leads interleaved rep by rep so box drift hits all
alike; then file -> totals through the device reader (bench.end_to_end's
leg).  Every lead's totals and a hit-matrix digest must be equal."""
from __future__ import annotations

import hashlib
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.file_io import read_batches
    from xspect2_amd.synth import make_genomes, make_reads

    leads = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,4").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    k, D, G, L = 21, 100, 4_000_000, 150
    dev = torch.device("cuda", 0)
    genomes = make_genomes(D, G, seed=42)
    bank = Bank.create_cobs(k, 7, [cobs_signature_size(G - k + 1, 7, 0.01)], D, [f"sp{i}" for i in range(D)])
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(D + 1, dtype=torch.int64, device=dev) * G
    s = torch.cuda.current_stream(dev)
    bank.build_device(g, genomes.size, go, D, torch.arange(D, dtype=torch.int32, device=dev), stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    N = 1_000_000
    reads, _ = make_reads(genomes, N, L, seed=42)
    d_seq = torch.from_numpy(reads.reshape(-1)).to(dev)
    sizes = [53_809, 107_351, 214_406, 428_811, 195_623, N]
    out = {"leads": leads, "reps": reps, "sizes": sizes, "calls": {}, "digests": {}}
    hits = torch.empty((N, D), dtype=torch.int32, device=dev)
    for lead in leads:  # parity: the same hits and totals whatever the lead
        bank.set_probe_options(lookup_lead=lead, cobs_part=2)
        d_off = torch.arange(N + 1, dtype=torch.int64, device=dev) * L
        tot = torch.zeros(D + 1, dtype=torch.int64, device=dev)
        bank.query_device(d_seq, N * L, d_off, N, 1, hits, None, tot, stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        out["digests"][lead] = hashlib.sha256(hits.cpu().numpy().tobytes() + tot.cpu().numpy().tobytes()).hexdigest()[:16]
    assert len(set(out["digests"].values())) == 1, out["digests"]
    del hits
    acc = {(lead, n): {"probe": [], "lookup": [], "bucket": [], "resolve": []} for lead in leads for n in sizes}
    for rep in range(reps):
        for lead in leads:
            bank.set_probe_options(lookup_lead=lead, cobs_part=1)
            for n in sizes:
                d_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
                tot = torch.zeros(D + 1, dtype=torch.int64, device=dev)
                for _ in range(2):
                    bank.query_device(d_seq, n * L, d_off, n, 1, None, None, tot, stream=s.cuda_stream)
                torch.cuda.synchronize(dev)
                bank.set_profiling(True)
                bank.probe_stats()
                bank.pass_stats()
                k_ = 5
                for _ in range(k_):
                    bank.query_device(d_seq, n * L, d_off, n, 1, None, None, tot, stream=s.cuda_stream)
                torch.cuda.synchronize(dev)
                launches, ms_tot, _ = bank.probe_stats()
                ps = bank.pass_stats()
                bank.set_profiling(False)
                a = acc[(lead, n)]
                a["probe"].append(ms_tot / launches)
                for p in ("lookup", "bucket", "resolve"):
                    a[p].append(ps[p][0] / max(1, launches))
        print(f"rep {rep} done", file=sys.stderr, flush=True)
    for (lead, n), a in acc.items():
        out["calls"].setdefault(str(lead), {})[str(n)] = {p: round(float(np.median(v)), 4) for p, v in a.items()}
    # the five windows' probe calls against one call: the per-call overhead the prefetch targets
    for lead in leads:
        c = out["calls"][str(lead)]
        five = sum(c[str(n)]["probe"] for n in sizes[:5])
        out.setdefault("five_vs_one", {})[str(lead)] = {"five_calls_ms": round(five, 4), "one_call_ms": c[str(N)]["probe"]}
    # file -> totals through the device reader (bench.end_to_end's device_reader_totals leg)
    tmp = Path(tempfile.mkdtemp(prefix="xs_lead_ab_"))
    fq = tmp / "reads.fastq"
    qual = b"I" * L
    with open(fq, "wb") as fh:
        for lo in range(0, N, 100_000):
            fh.write(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, reads[i].tobytes(), qual) for i in range(lo, min(N, lo + 100_000))))
    e2e = {str(lead): [] for lead in leads}
    for rep in range(reps + 1):
        for lead in leads:
            bank.set_probe_options(lookup_lead=lead, cobs_part=1)
            t = time.perf_counter()
            tot_all = np.zeros(D, dtype=np.uint64)
            for batch in read_batches(fq, device=bank.device):
                t_, _ = bank.query_totals(batch)
                tot_all += t_
            dt = (time.perf_counter() - t) * 1e3
            if rep:  # rep 0 warms the reader's pools
                e2e[str(lead)].append(dt)
    out["file_to_totals_ms"] = {k_: {"min": round(min(v), 3), "median": round(float(np.median(v)), 3)}
                                for k_, v in e2e.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
