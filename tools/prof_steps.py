"""Per-step breakdown of the timed region of a `rocprofv3 --kernel-trace` run of bench.py:
the last K W4A4Linear.forward steps (colmax, rank, quantizer, GEMM), their kernel times and
the idle gaps between kernels -- what the step time is made of.
    python tools/prof_steps.py <run_kernel_trace.csv> [K]"""
import csv
import statistics
import sys

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(name):
    for key in ("gemm_fq6", "gemm_f8", "quant_lc", "colmax", "rank_table", "rank_count",
                "lc_table", "colsum", "Cijk", "copyBuffer"):
        if key in name:
            return key
    return name.split("(")[0][-40:]


gemm = [i for i, r in enumerate(rows) if "gemm_fq6" in r["Kernel_Name"] or "gemm_f8_kernel" in r["Kernel_Name"]]
# the timed steps are the last K GEMMs of the forward loop (the CPU-baseline leg is off)
last = gemm[-K:]
start = last[0]
while start > 0 and short(rows[start - 1]["Kernel_Name"]) in ("quant_lc", "colmax", "rank_table", "rank_count", "lc_table", "colsum"):
    start -= 1
seg = rows[start:last[-1] + 1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = {}
gaps = []
for a, b in zip(seg, seg[1:]):
    gaps.append(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
for r in seg:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy.setdefault(short(r["Kernel_Name"]), []).append(d)
span = (t1 - t0) / 1e3
print(f"{K} steps: first kernel start -> last kernel end {span:.1f} us = {span / K:.1f} us/step")
for k, v in sorted(busy.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:12s} n={len(v):3d} avg {statistics.mean(v) / 1e3:8.2f} us  total/step {sum(v) / 1e3 / K:8.2f} us")
print(f"  gaps        n={len(gaps):3d} avg {statistics.mean(gaps) / 1e3:8.2f} us  total/step {sum(gaps) / 1e3 / K:8.2f} us"
      f"  (max {max(gaps) / 1e3:.1f} us)")
