"""Per-window table of one file -> totals pass from a rocprofv3 trace of
tools/e2e_trace.py (--kernel-trace --memory-copy-trace --output-format csv).

    python3 tools/e2e_trace_table.py <trace dir> <e2e_trace.py JSON line file> [--pass N]

Events are placed on the pass's own host clock (e2e_trace.py records each
pass's start and end on CLOCK_MONOTONIC, _RAW and BOOTTIME; the clock that
holds most trace events inside the passes is used).  Every kernel is a probe
kernel (cobs_*, part_*, probe_*, reduce_*, the scans on the bank's queue) or a
parse kernel (fx_*, fq_*, fa_*, the scans on the reader's queue); copies are
H2D or D2H.  Prints, for the chosen pass (default: the last), the merged
activity intervals in time order (ms from the pass start), then the busy time
of each class, their pairwise overlaps and the time nothing ran on the GPU.
"""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path


def _rows(path):
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


def _find(d: Path, suffix: str):
    f = sorted(d.rglob(f"*{suffix}"))
    return f[0] if f else None


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    return None


def load_events(d: Path):
    ev = []
    kt = _find(d, "kernel_trace.csv")
    rows = _rows(kt) if kt else []
    # the queue (or stream) that runs the probe's own kernels is the bank's
    qcol = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
    probe_q = {r.get(qcol) for r in rows if any(s in r["Kernel_Name"] for s in ("cobs_", "part_", "probe_"))}
    for r in rows:
        name = r["Kernel_Name"]
        if any(s in name for s in ("fx_", "fq_", "fa_")):
            cls = "parse"
        elif any(s in name for s in ("cobs_", "part_", "probe_", "reduce_partials", "units_", "scatter_units")):
            cls = "probe"
        else:  # scans, memsets: by queue
            cls = "probe" if r.get(qcol) in probe_q else "parse"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cls, name[:60], 0))
    mt = _find(d, "memory_copy_trace.csv")
    for r in (_rows(mt) if mt else []):
        direction = _col(r, "Direction", "Operation") or ""
        cls = "h2d" if "HOST_TO_DEVICE" in direction.upper() else "d2h" if "DEVICE_TO_HOST" in direction.upper() \
            else "copy"
        nbytes = int(_col(r, "Bytes", "Size", "Copy_Bytes") or 0)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cls, direction, nbytes))
    ev.sort()
    return ev


def merge(iv, gap=20_000):
    """Union of [s, e) intervals (ns), joining those less than `gap` apart."""
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1] + gap:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    d, meta_path = Path(sys.argv[1]), Path(sys.argv[2])
    which = int(sys.argv[sys.argv.index("--pass") + 1]) if "--pass" in sys.argv else -1
    meta = json.loads([ln for ln in meta_path.read_text().splitlines() if ln.startswith("{")][-1])
    ev = load_events(d)
    # the host clock that matches the trace
    best, best_n = None, -1
    for c, spans in meta["pass_clock_ns"].items():
        n = sum(1 for s, e, *_ in ev for a, b in spans if a <= s <= b)
        if n > best_n:
            best, best_n = c, n
    spans = meta["pass_clock_ns"][best]
    a, b = spans[which]
    p = [x for x in ev if a <= x[0] <= b]
    wall = (b - a) / 1e6
    print(f"trace {d}: {len(ev)} events; clock {best} ({best_n} events inside passes); pass {which} of "
          f"{len(spans)}: host wall {wall:.2f} ms, batches {meta['batches']}")
    by = {}
    for s, e, cls, name, nb in p:
        by.setdefault(cls, []).append((s, e, nb))
    rows = []
    for cls, iv in by.items():
        for s, e in merge([(s, e) for s, e, _ in iv]):
            nb = sum(x[2] for x in iv if s <= x[0] <= e)
            nk = sum(1 for x in iv if s <= x[0] <= e)
            rows.append((s, e, cls, nk, nb))
    rows.sort()
    print(f"{'start':>8} {'end':>8} {'ms':>6}  class  events  bytes")
    for s, e, cls, nk, nb in rows:
        print(f"{(s - a) / 1e6:8.2f} {(e - a) / 1e6:8.2f} {(e - s) / 1e6:6.2f}  {cls:<5} {nk:7d}  "
              f"{nb / 1e6:8.1f} MB" if nb else
              f"{(s - a) / 1e6:8.2f} {(e - a) / 1e6:8.2f} {(e - s) / 1e6:6.2f}  {cls:<5} {nk:7d}")
    busy = {cls: merge([(s, e) for s, e, _ in iv], 0) for cls, iv in by.items()}
    anyb = merge([iv for v in busy.values() for iv in v], 0)
    print("busy ms: " + ", ".join(f"{c} {length(v) / 1e6:.2f}" for c, v in sorted(busy.items())) +
          f"; any {length(anyb) / 1e6:.2f}; GPU idle inside the pass {wall - length(anyb) / 1e6:.2f}")
    cl = sorted(busy)
    for i in range(len(cl)):
        for j in range(i + 1, len(cl)):
            ov = length(intersect(busy[cl[i]], busy[cl[j]])) / 1e6
            print(f"overlap {cl[i]} & {cl[j]}: {ov:.2f} ms")
    if p:
        print(f"first event at {(p[0][0] - a) / 1e6:.2f} ms, last ends at {(max(x[1] for x in p) - a) / 1e6:.2f} ms")
    if "probe_alone" in meta:
        pa = meta["probe_alone"]
        print("probes alone (device-resident reads, host-timed): " +
              ", ".join(f"{c['reads']}: {c['ms']:.2f}" for c in pa) +
              f"; sum of the batches' {sum(c['ms'] for c in pa[:-1]):.2f} ms")


if __name__ == "__main__":
    main()
