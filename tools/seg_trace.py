"""Kernel durations per workload segment from a rocprofv3 --kernel-trace CSV.

A script that runs several workloads calls `mark()` between them (a torch.cuda._sleep
separator kernel) and prints the segment labels in order; `python tools/seg_trace.py
TRACE.csv LABELS.txt` then prints, per label, the median duration of each kernel name over
the segment's launches (first launch of each name skipped as warm-up when there are > 2).
"""
import csv
import statistics
import sys
from collections import OrderedDict


def mark():
    import torch
    torch.cuda.synchronize()
    torch.cuda._sleep(50_000)
    torch.cuda.synchronize()


def main(trace, labels_path):
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    segs, cur = [], []
    for r in rows:
        if "spin" in r[2] or "sleep" in r[2]:
            segs.append(cur)
            cur = []
        else:
            cur.append(r)
    segs.append(cur)
    labels = [l.rstrip("\n") for l in open(labels_path) if l.startswith("SEG ")]
    # segment i (after the i-th separator) belongs to label i
    for lab, seg in zip(labels, segs[1:]):
        by = OrderedDict()
        for s, e, n in seg:
            by.setdefault(n.split("(")[0].replace("void ", "")[:60], []).append((e - s) / 1e3)
        parts = []
        for n, d in by.items():
            d = d[1:] if len(d) > 2 else d
            parts.append(f"{n} x{len(d)} {statistics.median(d):.1f}")
        print(f"{lab[4:]:40s} | " + " | ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
