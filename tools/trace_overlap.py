#!/usr/bin/env python3
"""Overlap of two kernel families in a rocprofv3 --kernel-trace CSV (run anywhere, on the CSV):

    python tools/trace_overlap.py TRACE.csv --a k_wal_walk_sub,k_wal_resolve,k_wal_gather --b k_ragged_staged_pipe

Prints the last few dispatches with start / end relative to the first of them (and their queue),
then over the whole trace: the busy time of family A, of family B, the time both run at once, and
the wall span of the dispatches of either family.  The sliced WAL replay (wal.cc sliced_pass) is
meant to run slice 1's walk (A) beside slice 0's CRC batch (B): the overlap says whether it does.
"""
import argparse
import csv


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
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
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--a", required=True)
    p.add_argument("--b", required=True)
    p.add_argument("--show", type=int, default=16)
    a = p.parse_args()
    fa, fb = a.a.split(","), a.b.split(",")
    rows = list(csv.DictReader(open(a.csv)))
    q = "Queue_Id" if rows and "Queue_Id" in rows[0] else ("Stream_Id" if rows and "Stream_Id" in rows[0] else None)
    ev = []
    for r in rows:
        name = r["Kernel_Name"]
        fam = "A" if any(k in name for k in fa) else "B" if any(k in name for k in fb) else None
        short = name.replace("(anonymous namespace)::", "").replace("karma::engine::", "").replace("void ", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam, short.split("(")[0][:56], r.get(q, "")))
    ev.sort()
    t0 = ev[-a.show][0] if len(ev) >= a.show else ev[0][0]
    for s, e, fam, name, qq in ev[-a.show:]:
        print(f"{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} us  {fam or '-'}  q{qq:>3}  {name}")
    A = union([[s, e] for s, e, f, _, _ in ev if f == "A"])
    B = union([[s, e] for s, e, f, _, _ in ev if f == "B"])
    both = intersect(A, B)
    span = union([[s, e] for s, e, f, _, _ in ev if f])
    print(f"A busy {length(A) / 1e3:.1f} us, B busy {length(B) / 1e3:.1f} us, both at once {length(both) / 1e3:.1f} us "
          f"({100 * length(both) / max(1, min(length(A), length(B))):.1f} % of the smaller), "
          f"A or B {length(span) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
