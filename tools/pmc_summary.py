"""Summarise rocprofv3 --pmc passes (tools/gpu.sh pmc:KIND layout: <dir>/<kind>_<pass>/
run_counter_collection.csv) into one JSON per GEMM kind with the derived figures DESIGN.md
quotes, so every fraction can be recomputed from profiles/ alone.

    python tools/pmc_summary.py <pmc dir> <kind> <avg kernel us> <algorithmic bytes> <mfma cycles per inst> [out.json] [kernel-name substring, default gemm]
(avg kernel us <= 0: the median duration of the profiled dispatches)

Derivations (MI355X_MICROARCH.md: HBM / rocprofv3 sections):
  hbm_bytes      = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   (gfx950 FETCH_SIZE reads 1/2
                   of a wide coalesced stream; sizes are in KiB)
  clock_GHz      = GRBM_GUI_ACTIVE / 8 XCDs / kernel time       (profiled pass; reads low
                   against an unprofiled run)
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
  mfma_busy_chk  = SQ_INSTS_MFMA * cycles per MFMA (cross-check of the busy counter)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, match, durs=None):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match in r.get("Kernel_Name", ""):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                if durs is not None and "End_Timestamp" in r:
                    durs[r["Dispatch_Id"] + d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    root, kind, us, alg_bytes, cyc = sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4]), float(sys.argv[5])
    match = sys.argv[7] if len(sys.argv) > 7 else "gemm"
    c = {}
    durs = {}
    for d in sorted(glob.glob(os.path.join(root, f"{kind}_*"))):
        if os.path.isdir(d):
            c.update(load(d, match, durs))
    if us <= 0:  # the profiled dispatches' own mean duration (reads long against unprofiled runs)
        us = sorted(durs.values())[len(durs) // 2]
    t = us * 1e-6
    xcd_cycles = c["GRBM_GUI_ACTIVE"] / 8
    out = {
        "kind": kind, "avg_kernel_us": us, "counters_per_dispatch": c,
        "hbm_bytes_per_launch": 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024,
        "hbm_read_bytes": 2 * c["FETCH_SIZE"] * 1024, "hbm_write_bytes": c["WRITE_SIZE"] * 1024,
        "algorithmic_bytes": alg_bytes,
        "clock_GHz_profiled": xcd_cycles / t / 1e9,
        "mfma_busy": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * xcd_cycles),
        "mfma_busy_from_inst_count": c["SQ_INSTS_MFMA"] * cyc / (1024 * xcd_cycles),
        "valu_insts_per_mfma": c["SQ_INSTS_VALU"] / max(c["SQ_INSTS_MFMA"], 1),
        # VALU issue share: wave-instructions x 4 cycles over the SIMD-cycles of the launch
        "valu_issue_frac": c["SQ_INSTS_VALU"] * 4 / (1024 * xcd_cycles),
        "lds_bank_conflict_frac_of_lds_insts": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_INSTS_LDS", 1), 1),
        "l2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
        "wave_cycles_wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
        "wave_cycles_wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
    }
    out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / alg_bytes
    # the library build the counters describe (bench.py's pick_traffic matches on it); set
    # SQMP_PMC_LIB_SHA1 when summarising elsewhere than the tree that was profiled
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    out["lib_sha1"] = os.environ.get("SQMP_PMC_LIB_SHA1") or bench.lib_sha1()
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 6:
        open(sys.argv[6], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
