"""The end-to-end device path of the config-2 reads as a FASTQ file, batch
by batch on one thread (reader, then probe), for kernel traces:
    rocprofv3 --kernel-trace --stats -- python3 tools/e2e_seq.py [--reps N] [--totals|--hits]"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--hits", action="store_true")
    a = ap.parse_args()
    import torch
    from fx_dev_trace import write_fastq
    from xspect2_amd import file_io
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.synth import make_genomes

    p = Path("/tmp/xs_seq.fastq")
    write_fastq(p, 1_000_000)
    k, D, G = 21, 100, 4_000_000
    dev = torch.device("cuda", 0)
    genomes = make_genomes(D, G, seed=42)
    bank = Bank.create_cobs(k, 7, [cobs_signature_size(G - k + 1, 7, 0.01)], D, [f"sp{i}" for i in range(D)])
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(D + 1, dtype=torch.int64, device=dev) * G
    bank.build_device(g, genomes.size, go, D, torch.arange(D, dtype=torch.int32, device=dev),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    for rep in range(a.reps):
        time.sleep(0.3)
        t = time.perf_counter()
        for b in file_io.read_batches(p, device=0):
            bank.query(b, hit_dtype="auto") if a.hits else bank.query_totals(b)
        print(f"rep {rep}: {(time.perf_counter() - t) * 1e3:.2f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
