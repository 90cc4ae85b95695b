"""gpu_search.py - the reference-side ctypes binding of libxspect_hip.so.

This is the file a maintainer drops into the reference as
src/xspect/models/gpu_search.py.  It depends on
ctypes + numpy only: no torch, no xspect2_amd.  GpuSearch stands in for
cobs_index.Search (probabilistic_filter_model.py:389, :227) and for
rbloom.Bloom.load (probabilistic_single_filter_model.py:155-158).
Tested by tests/test_integration_stub.py.
"""
import ctypes as C
import os
from collections import namedtuple
import numpy as np

_lib = C.CDLL(os.environ.get("XSPECT_HIP_LIB", "libxspect_hip.so"))  # path or LD_LIBRARY_PATH
_lib.xs_bank_open.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
_lib.xs_query.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint64), C.c_uint64,
                          C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
_lib.xs_bank_doc_name.argtypes = [C.c_void_p, C.c_uint64]
_lib.xs_bank_doc_name.restype = C.c_char_p
_lib.xs_last_error.restype = C.c_char_p
_lib.xs_bank_close.argtypes = [C.c_void_p]
_lib.xs_bank_set_term_size.argtypes = [C.c_void_p, C.c_uint32]

class XsBankInfo(C.Structure):
    _fields_ = [("kind", C.c_int32), ("device", C.c_int32), ("term_size", C.c_uint32),
                ("num_hashes", C.c_uint32), ("canonicalize", C.c_uint32), ("reserved", C.c_uint32),
                ("num_docs", C.c_uint64), ("num_groups", C.c_uint64), ("page_size", C.c_uint64),
                ("signature_rows", C.c_uint64), ("bloom_bits", C.c_uint64),
                ("device_bytes", C.c_uint64), ("device_row_pitch", C.c_uint64)]
_lib.xs_bank_info.argtypes = [C.c_void_p, C.POINTER(XsBankInfo)]

COBS_CLASSIC, COBS_COMPACT, RBLOOM = 0, 1, 2
# cobs_index.SearchResult: the consumers read .doc_name and .score
# (probabilistic_filter_model.py:406-409, probabilistic_filter_mlst_model.py:377-380)
SearchResult = namedtuple("SearchResult", ["doc_name", "score"])

def _check(rc):
    if rc != 0:
        raise RuntimeError(_lib.xs_last_error().decode())

class GpuSearch:
    """Stands in for cobs_index.Search; search_batch() replaces a loop of search().
    rbloom files carry no k: pass term_size (the model JSON's "k") for RBLOOM."""
    def __init__(self, path, kind=COBS_CLASSIC, device=0, term_size=None):
        self.h = C.c_void_p()
        _check(_lib.xs_bank_open(str(path).encode(), kind, device, C.byref(self.h)))
        if term_size is not None:
            _check(_lib.xs_bank_set_term_size(self.h, term_size))
        info = XsBankInfo()
        _check(_lib.xs_bank_info(self.h, C.byref(info)))
        self.k, self.D = info.term_size, info.num_docs
        self.names = [(_lib.xs_bank_doc_name(self.h, d) or str(d).encode()).decode()
                      for d in range(self.D)]

    def search_batch(self, seqs, step=1, out=None):
        """seqs: list[str] -> (hits uint32 [n, D], num_kmers uint64 [n]).
        out: a reused C-contiguous uint32 [n, D] array; a serving loop passes
        one to skip what a fresh matrix costs the OS (faulting it in, and
        unmapping it when dropped: more than the query at 10^6 reads, DESIGN.md
        section 9c)."""
        data = [s.encode() for s in seqs]
        offs = np.zeros(len(data) + 1, np.uint64)
        offs[1:] = np.cumsum([len(b) for b in data])
        if out is not None and (out.shape != (len(data), self.D) or out.dtype != np.uint32
                                or not out.flags.c_contiguous):
            raise ValueError("out must be a C-contiguous uint32 [n, D] array")
        hits = np.empty((len(data), self.D), np.uint32) if out is None else out
        nk = np.empty(len(data), np.uint64)
        _check(_lib.xs_query(self.h, b"".join(data),
                             offs.ctypes.data_as(C.POINTER(C.c_uint64)), len(data), step,
                             hits.ctypes.data_as(C.POINTER(C.c_uint32)),
                             nk.ctypes.data_as(C.POINTER(C.c_uint64))))
        return hits, nk

    def search(self, seq, step=1):
        """cobs_index.Search.search(): every doc as SearchResult(doc_name, score),
        score descending (ties by doc index; COBS's own tie order is unpinned)."""
        row = self.search_batch([seq], step)[0][0]
        order = sorted(range(self.D), key=lambda d: (-int(row[d]), d))
        return [SearchResult(self.names[d], int(row[d])) for d in order]

    def __del__(self):
        if getattr(self, "h", None):
            _lib.xs_bank_close(self.h)
