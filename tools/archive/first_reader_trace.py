"""First device reader of a process, traced (XSPECT2_AMD_FASTX_TRACE): where its one-time cost goes."""
import os, sys, time
os.environ["XSPECT2_AMD_FASTX_TRACE"] = "1"
sys.path.insert(0, "/root/repo")
from xspect2_amd import _lib
from xspect2_amd.bank import Bank
import numpy as np
_lib.load(); _lib.device_count()
tiny = Bank.create_cobs(21, 7, [1001], 100); tiny.upload(np.zeros(tiny.payload_bytes(), np.uint8)); tiny.close()
from pathlib import Path
fq = Path("/tmp/fr.fq")
fq.write_bytes(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, b"ACGT" * 37 + b"AC", b"I" * 150) for i in range(1000)))
from xspect2_amd.file_io import read_batches
for k in range(2):
    t = time.perf_counter()
    print(f"--- reader {k} at {time.monotonic()*1e3:.2f}", file=sys.stderr, flush=True)
    n = sum(b.n for b in read_batches(fq, 1 << 20, device=0))
    print(f"--- reader {k} {n} reads {(time.perf_counter()-t)*1e3:.2f} ms", file=sys.stderr, flush=True)
