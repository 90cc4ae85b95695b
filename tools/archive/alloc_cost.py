"""Cost of hipHostMalloc / hipMalloc by size, first touch excluded (diagnostics, GPU)."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
out = {}
for mb in (1, 4, 16, 64, 256):
    n = mb << 20
    th, td = [], []
    for _ in range(3):
        p = ctypes.c_void_p()
        t = time.perf_counter(); assert hip.hipHostMalloc(ctypes.byref(p), n, 0) == 0; th.append(time.perf_counter() - t)
        hip.hipHostFree(p)
        t = time.perf_counter(); assert hip.hipMalloc(ctypes.byref(p), n) == 0; td.append(time.perf_counter() - t)
        hip.hipFree(p)
    out[f"{mb}MiB"] = {"hipHostMalloc_ms": round(min(th) * 1e3, 3), "hipMalloc_ms": round(min(td) * 1e3, 3)}
print(json.dumps(out))
