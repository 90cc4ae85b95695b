"""PackedIds (read ids kept as the reader's buffer + offsets) against the
list-of-strings semantics it replaces (CPU): json.dumps quoting
(xs_ids_json_quote), duplicate detection (xs_ids_has_duplicates),
membership, slicing, concatenation, and MatrixResult.save writing the same
bytes with packed or listed ids (result.py:151-202 via json.dumps)."""
from __future__ import annotations

import json

import numpy as np
import pytest

from xspect2_amd.packing import PackedIds
from xspect2_amd.result import MatrixResult, _json_packed


def _ids(rng, n, alphabet):
    out = []
    for _ in range(n):
        L = int(rng.integers(0, 12))
        out.append("".join(rng.choice(alphabet, L)))
    return out


ASCII = list("abcXYZ019_-.:|/ ") + ['"', "\\", "\n", "\r", "\t", "\b", "\f", "\x00", "\x01", "\x1f", "\x7f"]


@pytest.mark.parametrize("seed", range(5))
def test_json_quote_and_duplicates_match_python(seed):
    rng = np.random.default_rng(seed)
    ids = _ids(rng, 3000, ASCII)
    if seed % 2:
        ids = list(dict.fromkeys(ids))  # no repeats
    p = PackedIds.of(ids)
    assert p.is_ascii and p == ids and len(p) == len(ids)
    assert p.json_packed()[0] == _json_packed(ids)[0]
    assert np.array_equal(p.json_packed()[1], _json_packed(ids)[1])
    assert p.has_duplicates() == (len(set(ids)) != len(ids))


def test_duplicates_over_threads():
    """xs_ids_has_duplicates at sizes that use its threads (hashing split over
    up to 16 threads, 256 hash buckets searched in parallel): 300 k distinct
    ids, then one repeat placed first/last, across the threads' ranges, an
    empty id twice, and ids that are prefixes of each other."""
    base = [f"read_{i}" for i in range(300_000)]
    assert not PackedIds.of(base).has_duplicates()
    assert not PackedIds.of(base + [f"read_{i}x" for i in range(1000)] + [""]).has_duplicates()
    for a, b in ((0, 299_999), (10, 150_000), (70_000, 70_001), (299_998, 5)):
        ids = list(base)
        ids[b] = ids[a]
        assert PackedIds.of(ids).has_duplicates(), (a, b)
    assert PackedIds.of(base + ["", ""]).has_duplicates()
    assert PackedIds.of([""] + base + [""]).has_duplicates()


def test_non_ascii_ids_fall_back_to_python():
    ids = ["r1", "é", "ü∑", "r1x", "\U0001F600"]
    p = PackedIds.of(ids)
    assert not p.is_ascii and p.tolist() == ids
    assert p.json_packed()[0] == b"".join(json.dumps(s).encode() for s in ids)
    assert not p.has_duplicates() and PackedIds.of(ids + ["é"]).has_duplicates()
    raw = PackedIds(b"a\xffb\xfe", np.array([0, 2, 4], dtype=np.uint64))  # invalid UTF-8: replacement chars
    assert raw.tolist() == [b"a\xff".decode("utf-8", "replace"), b"b\xfe".decode("utf-8", "replace")]


def test_membership_slicing_concat():
    ids = ["total1", "xtotal", "tot", "al", "total", "", "r7"]
    p = PackedIds.of(ids)
    for s in ids + ["otal", "totalx", "to", "r", "7", "missing"]:
        assert (s in p) == (s in ids), s
    assert "total" not in PackedIds.of(["total1", "xtotal", "tota", "ltotal"])
    assert "" not in PackedIds.of(["a", "b"]) and "" in PackedIds.of(["a", "", "b"])
    assert p[2:5] == ids[2:5] and p[::2] == ids[::2] and p[-1] == ids[-1] and list(p) == ids
    q = PackedIds.concat([p[0:3], p[3:], PackedIds.of(["z"])])
    assert q == ids + ["z"] and q.json_packed()[0] == _json_packed(ids + ["z"])[0]
    assert PackedIds.concat([PackedIds.of([])]) == []


@pytest.mark.parametrize("dup", [False, True])
def test_matrix_result_with_packed_ids_writes_the_same_json(tmp_path, dup):
    rng = np.random.default_rng(3)
    n, D = 500, 7
    ids = [f"read_{i % 300 if dup else i}\t\"q\"" for i in range(n)]
    hits = rng.integers(0, 50, (n, D)).astype(np.uint8)
    nk = rng.integers(50, 60, n).astype(np.uint64)
    labels = [f"L{d}" for d in range(D)]
    a = MatrixResult("slug", ids, labels, hits, nk, input_source="x.fq")
    b = MatrixResult("slug", PackedIds.of(ids), labels, hits, nk, input_source="x.fq")
    assert isinstance(b.ids, PackedIds) != dup  # repeated ids collapse through the list path
    a.save(tmp_path / "a.json")
    b.save(tmp_path / "b.json")
    assert (tmp_path / "a.json").read_bytes() == (tmp_path / "b.json").read_bytes()
    assert b.get_filter_mask("L3", 0.5) == a.get_filter_mask("L3", 0.5)
    with pytest.raises(ValueError, match="reserved"):
        MatrixResult("slug", PackedIds.of(["a", "total"]), ["x"], np.zeros((2, 1), np.uint8), np.ones(2))


def test_hash128_is_xxh64_with_two_seeds():
    """xs_ids_hash128 = python-xxhash's XXH64 of each id's bytes, seeds 0 and
    0x27D4EB2F165667C5 (lengths 0..80 cover every tail path, non-ASCII too)."""
    import xxhash
    from xspect2_amd.packing import PackedIds
    rng = np.random.default_rng(3)
    ids = [bytes(rng.integers(0, 256, n, dtype=np.uint8)).decode("latin-1") for n in range(81)] + ["read_1", "é"]
    p = PackedIds.of(ids)
    h = p.hash128()
    for i, s in enumerate(ids):
        b = s.encode("utf-8")
        assert int(h[i, 0]) == xxhash.xxh64_intdigest(b, 0)
        assert int(h[i, 1]) == xxhash.xxh64_intdigest(b, 0x27D4EB2F165667C5)


def test_take_keeps_the_selected_ids_packed():
    from xspect2_amd.packing import PackedIds
    ids = ["a", "", "read_22", "x" * 40, "é", "b"]
    p = PackedIds.of(ids)
    for idx in ([], [0], [5, 0, 2], [1, 1, 3], list(range(6))):
        t = p.take(np.array(idx, dtype=np.int64))
        assert isinstance(t, PackedIds) and t.tolist() == [ids[i] for i in idx]


def test_drop_keeps_every_other_id_in_order():
    """PackedIds.drop (the repeated-id resolution of sharded jobs) equals the
    list without the dropped positions: none, some, repeated indices, all."""
    import numpy as np
    from xspect2_amd.packing import PackedIds
    rng = np.random.default_rng(3)
    ids = [f"read_{i}" + "x" * int(rng.integers(0, 5)) for i in range(500)] + ["", "é", ""]
    p = PackedIds.of(ids)
    for drop in ([], [0], [502], [5, 5, 7, 499, 0], list(range(0, 503, 3)), list(range(503))):
        keep = [s for i, s in enumerate(ids) if i not in set(drop)]
        q = p.drop(np.array(drop, dtype=np.int64))
        assert q.tolist() == keep and len(q) == len(keep)
        assert q.tolist() == p.take(np.array([i for i in range(503) if i not in set(drop)], dtype=np.int64)).tolist()


def test_u64_member_mask_matches_isin():
    """xs_u64_member_mask (the owner's candidate search of a sharded job) =
    numpy's isin, for random keys, repeats in the set, 0 and 2^64-1."""
    import numpy as np
    from xspect2_amd._lib import check, load
    rng = np.random.default_rng(9)
    keys = rng.integers(0, 1 << 62, 200_000, dtype=np.int64).view(np.uint64)
    keys[:4] = [0, np.uint64(2**64 - 1), 5, 5]
    for m in (0, 1, 7, 5000):
        st = np.concatenate([keys[rng.integers(0, keys.size, m)], rng.integers(0, 1 << 62, m, dtype=np.int64)
                             .view(np.uint64)]) if m else np.zeros(0, np.uint64)
        if m:
            st[:2] = [0, np.uint64(2**64 - 1)]
        st = np.ascontiguousarray(st)
        out = np.empty(keys.size, dtype=np.uint8)
        check(load().xs_u64_member_mask(keys.ctypes.data, keys.size, st.ctypes.data if st.size else None, st.size,
                                        out.ctypes.data))
        assert np.array_equal(out.astype(bool), np.isin(keys, st))


def test_c_abi_turns_a_failed_host_allocation_into_an_error_code():
    """No C++ exception leaves the library (xs::guard around every entry
    point): a set of 2^55 keys needs a 2^59-byte hash table, whose allocation
    fails before the set is read; the call returns XS_ERR_NOMEM with a
    message instead of ending the process."""
    import numpy as np
    from xspect2_amd import _lib
    keys = np.zeros(1, dtype=np.uint64)
    one = np.zeros(1, dtype=np.uint64)  # stands in for the set: never read
    out = np.empty(1, dtype=np.uint8)
    rc = _lib.load().xs_u64_member_mask(keys.ctypes.data, 1, one.ctypes.data, 1 << 55, out.ctypes.data)
    assert rc == _lib.XS_ERR_NOMEM
    assert b"allocation" in _lib.load().xs_last_error()
    # the library still works afterwards
    _lib.check(_lib.load().xs_u64_member_mask(keys.ctypes.data, 1, one.ctypes.data, 1, out.ctypes.data))
    assert out[0] == 1


def test_index_finds_the_first_equal_id():
    """PackedIds.index (the sharded totals' search for a read named
    "misclassified") = list.index, also for prefixes, suffixes and repeats."""
    import pytest
    from xspect2_amd.packing import PackedIds
    ids = ["amisclassified", "misclassifiedx", "mis", "misclassified", "", "misclassified", "é"]
    p = PackedIds.of(ids[:-1])
    for s in ("misclassified", "mis", "", "amisclassified", "misclassifiedx"):
        assert p.index(s) == ids.index(s)
    with pytest.raises(ValueError):
        p.index("classified")
    assert PackedIds.of(ids).index("é") == 6


def test_host_workers_from_threads_and_after_fork():
    """The library's persistent host workers (xs_pool.cpp) behind the threaded
    id passes: 8 Python threads hashing 1 M-id batches at once through the
    C ABI (ctypes releases the GIL) all get the one-thread answer; a forked
    child, which has none of the parent's workers, gets it too."""
    import os
    import threading

    from xspect2_amd.packing import PackedIds
    ids = PackedIds.of([f"read_{i}" for i in range(1_000_000)])
    want = ids.hash128()  # threaded: 1 M ids / 2^16 per thread
    got, errs = [None] * 8, []

    def work(i):
        try:
            got[i] = ids.hash128()
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs and all(np.array_equal(g, want) for g in got)
    pid = os.fork()
    if pid == 0:  # child: any failure is its exit code
        ok = False
        try:
            ok = bool(np.array_equal(ids.hash128(), want) and ids.has_duplicates() is False)
        finally:
            os._exit(0 if ok else 1)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
