"""What page-locked host memory costs to set up on this box (the first call
of a process pays it: the reader's 128 MiB text ring, the host-output
staging slots; DESIGN §8 f1 "First call"), and whether it copies as fast:

  malloc_pinned     hipHostMalloc(n)
  register_4k       mmap + memset (1 thread) + hipHostRegister
  register_thp8     mmap + madvise(MADV_HUGEPAGE) + memset (8 threads) + hipHostRegister
  h2d_*             one n-byte hipMemcpy host -> device from that memory, best of 5
  free_*            hipHostFree / hipHostUnregister + munmap

for n = 32 and 128 MiB, best of 3 setups each.  One JSON line.
"""
from __future__ import annotations

import ctypes
import json
import mmap
import threading
import time

hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
libc = ctypes.CDLL(None)
libc.memset.restype = ctypes.c_void_p
libc.memset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
for f in ("hipHostMalloc", "hipMalloc"):
    getattr(hip, f).argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t] + (
        [ctypes.c_uint] if f == "hipHostMalloc" else [])
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
H2D = 1
MADV_HUGEPAGE = 14


def ok(rc):
    if rc != 0:
        raise RuntimeError(f"HIP error {rc}")


def ms(t0):
    return (time.perf_counter() - t0) * 1e3


def fill(p, n, threads):
    per = (n + threads - 1) // threads
    th = [threading.Thread(target=libc.memset, args=(p + i * per, 0, min(per, n - i * per)))
          for i in range(threads) if i * per < n]
    for x in th:
        x.start()
    for x in th:
        x.join()


def h2d(dev, p, n):
    """(first copy, best of the next four) in ms"""
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        ok(hip.hipMemcpy(dev, p, n, H2D))
        ts.append(ms(t0))
    return ts[0], min(ts[1:])


def run(n, dev):
    out = {}
    # hipHostMalloc
    setup, free, copy = [], [], []
    for _ in range(3):
        p = ctypes.c_void_p()
        t0 = time.perf_counter()
        ok(hip.hipHostMalloc(ctypes.byref(p), n, 0))
        setup.append(ms(t0))
        copy.append(h2d(dev, p, n))
        t0 = time.perf_counter()
        ok(hip.hipHostFree(p))
        free.append(ms(t0))
    out["malloc_pinned"] = {"setup_ms": min(setup), "h2d_first_ms": min(c[0] for c in copy),
                            "h2d_ms": min(c[1] for c in copy), "free_ms": min(free)}
    for name, huge, threads in (("register_4k", False, 1), ("register_thp8", True, 8)):
        setup, free, copy, parts = [], [], [], []
        for _ in range(3):
            t0 = time.perf_counter()
            raw = libc.mmap(None, n + (2 << 20), 3, 0x22, -1, 0)  # PROT_READ|WRITE, MAP_PRIVATE|ANONYMOUS
            p = (raw + (2 << 20) - 1) // (2 << 20) * (2 << 20)
            if huge:
                libc.madvise(p, n, MADV_HUGEPAGE)
            fill(p, n, threads)
            t1 = time.perf_counter()
            ok(hip.hipHostRegister(p, n, 0))
            setup.append(ms(t0))
            parts.append({"touch_ms": (t1 - t0) * 1e3, "register_ms": ms(t1)})
            copy.append(h2d(dev, p, n))
            t0 = time.perf_counter()
            ok(hip.hipHostUnregister(p))
            libc.munmap(raw, n + (2 << 20))
            free.append(ms(t0))
        i = setup.index(min(setup))
        out[name] = {"setup_ms": setup[i], **parts[i], "h2d_first_ms": min(c[0] for c in copy),
                     "h2d_ms": min(c[1] for c in copy), "free_ms": min(free)}
    return out


def main():
    ok(hip.hipSetDevice(0))
    dev = ctypes.c_void_p()
    ok(hip.hipMalloc(ctypes.byref(dev), 128 << 20))
    res = {f"{mb}MiB": run(mb << 20, dev) for mb in (32, 128)}
    ok(hip.hipFree(dev))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
