"""Start-up costs of a one-shot `xspect classify` process on this box (the
reference's CLI runs one process per input): the package import, loading
libxspect_hip.so, the first HIP call, the first kernel launch (a tiny bank's
repack: the library's code object goes to the GPU), a bank file opening onto
the device and the first small query, each timed in a fresh child process (so nothing is
warm but the page cache).  One JSON line.

    python tools/cli_probe.py
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]

CHILD = r'''
import json, sys, time
t = {}
t0 = time.perf_counter()
sys.path.insert(0, %r)
import numpy as np
t["import_numpy_s"] = time.perf_counter() - t0
t1 = time.perf_counter()
from xspect2_amd import _lib
from xspect2_amd.bank import Bank
from xspect2_amd import probabilistic_filter_model, result, file_io
t["import_package_s"] = time.perf_counter() - t1
t1 = time.perf_counter()
lib = _lib.load()
t["load_library_s"] = time.perf_counter() - t1
t1 = time.perf_counter()
n = _lib.device_count()
t["first_hip_call_s"] = time.perf_counter() - t1
t1 = time.perf_counter()
tiny = Bank.create_cobs(21, 7, [1001], 100)
tiny.upload(np.zeros(tiny.payload_bytes(), np.uint8))  # the first kernel launch (the repack)
tiny.close()
t["first_kernel_s"] = time.perf_counter() - t1
fq = sys.argv[2]
from xspect2_amd.file_io import read_batches
for name in ("first_device_reader_s", "second_device_reader_s"):  # the parse kernels' module, then warm
    t1 = time.perf_counter()
    nb = sum(bt.n for bt in read_batches(fq, 1 << 20, device=0))
    t[name] = time.perf_counter() - t1
path = sys.argv[1]
if path != "-":
    t1 = time.perf_counter()
    b = Bank.open(path, _lib.XS_BANK_COBS_CLASSIC, device=0)
    t["bank_open_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    b.query([b"ACGT" * 40])
    t["first_query_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    b.query([b"ACGT" * 40])
    t["second_query_s"] = time.perf_counter() - t1
    b.close()
t["total_s"] = time.perf_counter() - t0
print(json.dumps(t))
'''


def main():
    import numpy as np
    sys.path.insert(0, str(ROOT))
    path = Path("/tmp/xs_cli_probe.cobs_classic")
    # a small bank file made in a child process (this one stays free of HIP)
    make = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np\n"
            "from xspect2_amd.bank import Bank\n"
            "b = Bank.create_cobs(21, 7, [2_000_003], 100, [f'd{i}' for i in range(100)])\n"
            "b.upload(np.random.default_rng(1).integers(0, 256, b.payload_bytes(), dtype=np.uint8))\n"
            "b.save(%r)\n" % (str(ROOT), str(path)))
    subprocess.run([sys.executable, "-c", make], check=True)
    fq = Path("/tmp/xs_cli_probe.fq")
    fq.write_bytes(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, b"ACGT" * 37 + b"AC", b"I" * 150) for i in range(1000)))
    runs = []
    for _ in range(3):
        r = subprocess.run([sys.executable, "-c", CHILD % str(ROOT), str(path), str(fq)], check=True,
                           capture_output=True, text=True)
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    path.unlink()
    fq.unlink()
    best = {k: min(r[k] for r in runs) for k in runs[0]}
    print(json.dumps({"runs": runs, "best": best, "bank_file_mb": 2_000_003 * 13 / 1e6}), flush=True)


if __name__ == "__main__":
    main()
