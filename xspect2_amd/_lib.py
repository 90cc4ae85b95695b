"""ctypes binding of libxspect_hip.so (include/xspect_hip.h).

The library is built in-tree (``xspect2_amd/libxspect_hip.so``) by
``xspect2_amd.build.build_library()``.  There is no CPU fallback: if the shared
object is missing or cannot be loaded, importing this module raises.
"""
from __future__ import annotations

import ctypes
import importlib.util
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
SO_PATH = PKG / "libxspect_hip.so"

XS_OK = 0
XS_ERR_ARG = -1
XS_ERR_IO = -2
XS_ERR_FORMAT = -3
XS_ERR_HIP = -4
XS_ERR_UNSUPPORTED = -5
XS_ERR_NOMEM = -6
XS_ERR_INTERNAL = -7

XS_BANK_COBS_CLASSIC = 0
XS_BANK_COBS_COMPACT = 1
XS_BANK_RBLOOM = 2
XS_PATH_GATHER = 0
XS_PATH_PARTITIONED = 1

XS_BEST_AMBIGUOUS = 0xFFFFFFFF

XS_FASTX_FASTA = 1
XS_FASTX_FASTQ = 2
XS_FASTX_PINNED = 1


class XsError(RuntimeError):
    """A failed libxspect_hip call (message from xs_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[xs {code}] {msg}")
        self.code = code


class BankInfo(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("term_size", ctypes.c_uint32),
        ("num_hashes", ctypes.c_uint32),
        ("canonicalize", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("num_docs", ctypes.c_uint64),
        ("num_groups", ctypes.c_uint64),
        ("page_size", ctypes.c_uint64),
        ("signature_rows", ctypes.c_uint64),
        ("bloom_bits", ctypes.c_uint64),
        ("device_bytes", ctypes.c_uint64),
        ("device_row_pitch", ctypes.c_uint64),
    ]


class ProbeOptions(ctypes.Structure):
    """xs_probe_options_t: path selection of one bank handle (defaults = production)."""
    _fields_ = [
        ("cobs_part", ctypes.c_int32),
        ("bloom_part", ctypes.c_int32),
        ("workspace_mib", ctypes.c_uint32),
        ("small_calls", ctypes.c_int32),
    ]


class FastxBatch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("seq_bytes", ctypes.c_uint64),
        ("seqs", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("ids", ctypes.c_void_p),
        ("id_offsets", ctypes.c_void_p),
        ("text_offset", ctypes.c_uint64),
        ("text_bytes", ctypes.c_uint64),
        ("descs", ctypes.c_void_p),
        ("desc_offsets", ctypes.c_void_p),
    ]


class FastxDBatch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("seq_bytes", ctypes.c_uint64),
        ("seqs", ctypes.c_void_p),       # device
        ("offsets", ctypes.c_void_p),    # device
        ("host_offsets", ctypes.c_void_p),
        ("max_len", ctypes.c_uint64),
        ("ids", ctypes.c_void_p),
        ("id_offsets", ctypes.c_void_p),
        ("descs", ctypes.c_void_p),
        ("desc_offsets", ctypes.c_void_p),
        ("text_offset", ctypes.c_uint64),
        ("text_bytes", ctypes.c_uint64),
        ("parsed_on_device", ctypes.c_int),
        ("host_ready", ctypes.c_void_p),
    ]


_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_int = ctypes.c_int
_pp = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); every symbol of include/xspect_hip.h
SIGNATURES = {
    "xs_version": (_int, []),
    "xs_build_id": (ctypes.c_char_p, []),
    "xs_last_error": (ctypes.c_char_p, []),
    "xs_device_count": (_int, [ctypes.POINTER(_int)]),
    "xs_bank_open": (_int, [ctypes.c_char_p, _int, _int, _pp]),
    "xs_bank_open_docs": (_int, [ctypes.c_char_p, _int, _u64, _u64, _pp]),
    "xs_bank_create_cobs": (_int, [_int, _int, _u32, _u32, _u64, _u64, _u64, _vp, _vp, _pp]),
    "xs_bank_create_bloom": (_int, [_int, _u32, _u64, _u32, _pp]),
    "xs_bank_build": (_int, [_vp, _vp, _vp, _vp, _u64]),
    "xs_bank_build_device": (_int, [_vp, _vp, _u64, _vp, _vp, _u64, _vp]),
    "xs_bank_save": (_int, [_vp, ctypes.c_char_p]),
    "xs_bank_download": (_int, [_vp, _vp, _u64]),
    "xs_bank_upload": (_int, [_vp, _vp, _u64]),
    "xs_bank_set_term_size": (_int, [_vp, _u32]),
    "xs_bank_info": (_int, [_vp, ctypes.POINTER(BankInfo)]),
    "xs_bank_signature_sizes": (_int, [_vp, _vp, _u64]),
    "xs_bank_doc_name": (ctypes.c_char_p, [_vp, _u64]),
    "xs_query": (_int, [_vp, _vp, _vp, _u64, _u32, _vp, _vp]),
    "xs_query_hits": (_int, [_vp, _vp, _vp, _u64, _u32, _vp, _int, _vp]),
    "xs_query_hits_device": (_int, [_vp, _vp, _u64, _vp, _u64, _u64, _u32, _vp, _int, _vp, _vp]),
    "xs_memcpy_to_host": (_int, [_vp, _vp, _u64]),
    "xs_memcpy_device": (_int, [_vp, _vp, _u64, _vp]),
    "xs_host_alloc": (_int, [_u64, _pp]),
    "xs_host_free": (None, [_vp]),
    "xs_query_totals": (_int, [_vp, _vp, _vp, _u64, _u32, _vp, _vp]),
    "xs_query_device": (_int, [_vp, _vp, _u64, _vp, _u64, _u32, _vp, _vp, _vp, _vp]),
    "xs_query_best": (_int, [_vp, _vp, _vp, _u64, _u32, _vp, _vp, _vp, _vp]),
    "xs_gather_reads_device": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "xs_best_device": (_int, [_vp, _u64, _u64, _vp, _vp, _vp]),
    "xs_mlst_sum": (_int, [_vp, _vp, _vp, _u64, _u64, _u32, _vp]),
    "xs_mlst_query": (_int, [_vp, _vp, _vp, _u64, _u64, _vp, _u64, _u32, _u32, _vp, _vp, _vp, _vp]),
    "xs_bank_set_profiling": (_int, [_vp, _int]),
    "xs_bank_last_probe_ms": (_int, [_vp, ctypes.POINTER(ctypes.c_float)]),
    "xs_bank_probe_stats": (_int, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_float)]),
    "xs_bank_probe_rows": (_int, [_vp, ctypes.POINTER(_u64)]),
    "xs_bank_pass_stats": (_int, [_vp, _vp, _vp]),
    "xs_bank_probe_path": (_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "xs_bank_set_probe_options": (_int, [_vp, ctypes.POINTER(ProbeOptions)]),
    "xs_bank_get_probe_options": (_int, [_vp, ctypes.POINTER(ProbeOptions)]),
    "xs_bank_workspace_bytes": (_int, [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "xs_bank_close": (None, [_vp]),
    "xs_write_result_sections": (_int, [ctypes.c_char_p, _u64, _u64, _vp, _int, _vp, ctypes.c_char_p, _vp,
                                        ctypes.c_char_p, _vp, _vp, _vp, _u64, _vp, _int]),
    "xs_ids_json_quote": (_int, [ctypes.c_char_p, _vp, _u64, _vp, _u64, _vp]),
    "xs_ids_has_duplicates": (_int, [ctypes.c_char_p, _vp, _u64, ctypes.POINTER(_int)]),
    "xs_ids_hash128": (_int, [ctypes.c_char_p, _vp, _u64, _vp]),
    "xs_u64_member_mask": (_int, [_vp, _u64, _vp, _u64, _vp]),
    "xs_fastx_open": (_int, [ctypes.c_char_p, _int, _int, _int, _pp]),
    "xs_fastx_open_range": (_int, [ctypes.c_char_p, _int, _int, _int, _u32, _u32, _pp]),
    "xs_fastx_next": (_int, [_vp, _u64, ctypes.POINTER(FastxBatch)]),
    "xs_fastx_close": (None, [_vp]),
    "xs_fastx_open_device": (_int, [ctypes.c_char_p, _int, _int, _int, _u32, _u32, _pp]),
    "xs_fastx_next_device": (_int, [_vp, _u64, ctypes.POINTER(FastxDBatch)]),
    "xs_fastx_wait_host": (_int, [ctypes.POINTER(FastxDBatch)]),
    "xs_write_fasta": (_int, [ctypes.c_char_p, _int, _vp, _vp, ctypes.c_char_p, _vp, _vp, _u64, _u32]),
}

_LIB = None


def _preload_hip_runtime() -> None:
    """One HIP runtime per process, without importing torch.

    torch's ROCm build carries its own libamdhip64 (SONAME libamdhip64.so.7)
    and its libtorch_hip asks for it by file name, so a process that loaded
    /opt/rocm's copy first (through this library's RUNPATH) would load a
    second runtime when torch is imported, and device pointers would not pass
    between them.  Loading torch's copy first (RTLD_GLOBAL) makes both this
    library (by SONAME) and a later `import torch` (the same file) use it.
    Importing torch itself for that cost a one-shot `xspect classify` process
    1.2 s; the runtime alone is ~20 ms (tools/cli_probe.py,
    profiles/r05u_cli*.json).  Without torch, /opt/rocm's runtime is used."""
    if "torch" in sys.modules:
        return  # torch has loaded its runtime already
    try:
        spec = importlib.util.find_spec("torch")  # locates, does not import
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    for root in spec.submodule_search_locations:
        hip = Path(root) / "lib" / "libamdhip64.so"
        if hip.exists():
            try:
                ctypes.CDLL(str(hip), mode=ctypes.RTLD_GLOBAL)
            except OSError:  # an unusable torch install: this library's own runtime then
                pass
            return


def load() -> ctypes.CDLL:
    """Load the in-tree shared library (raises if it is missing)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = SO_PATH
    if not path.exists():
        raise ImportError(
            f"{SO_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the probe path has no CPU fallback)")
    _preload_hip_runtime()
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int) -> None:
    if rc != XS_OK:
        msg = load().xs_last_error()
        raise XsError(rc, msg.decode() if msg else "unknown error")


def build_id() -> str:
    """The loaded library's build id (xspect2_amd.build.source_id of its sources)."""
    return load().xs_build_id().decode()


def device_count() -> int:
    n = _int(0)
    rc = load().xs_device_count(ctypes.byref(n))
    return n.value if rc == XS_OK else 0
