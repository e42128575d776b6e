"""Summarise one tools/profile_round.sh run into the committed profile files.

    python tools/traffic_summary.py gpurun_out/prof_TAG profiles/TAG [K T [c3|c2|c5 [traffic file name]]]

Reads the kernel-trace stats and the PMC passes (each counter in its own
rocprofv3 run, as the MI355X guide prescribes), applies the measured gfx950
calibration (tools/calib_fetch.hip: the same 8 B/lane [T][K][2] row pattern
with a known byte count; FETCH_SIZE reports that pattern at ~0.5x its true
bytes, WRITE_SIZE at 1.0x) and writes:

  profiles/TAG/kernel_stats.csv      rocprofv3 --kernel-trace --stats summary
  profiles/TAG/pmc_*.csv.gz          the counter CSVs (one per pass), gzipped
  profiles/TAG/sq_counters.json      SQ issue / wait summary
  profiles/traffic.json              HBM bytes and VALU instructions per rollout launch (read by bench.py)
"""
import csv
import gzip
import json
import os
import re
import shutil
import sys

import numpy as np


def counters(path, name_filter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if name_filter not in row["Kernel_Name"]:
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return vals


def main():
    src, dst = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    T = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    workload = sys.argv[5] if len(sys.argv) > 5 else "c3"
    bps = 28 if workload == "c5" else 8     # algorithmic noise bytes per state-step
    kpat = "chain_rollout_kernel" if workload == "c5" else "rollout_kernel"
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for p in ("fetch", "write", "cfetch", "cwrite", "sq", "grbm"):
        f = os.path.join(src, p, "p_counter_collection.csv")
        if os.path.exists(f):   # kept gzipped: the raw counter rows are large and only the summaries are cited
            with open(f, "rb") as fi, gzip.open(os.path.join(dst, f"pmc_{p}.csv.gz"), "wb", compresslevel=9) as fo:
                shutil.copyfileobj(fi, fo)
    avg_ns = None
    with open(os.path.join(src, "stats", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            if kpat in row["Name"] and (workload == "c5" or "chain" not in row["Name"]):
                avg_ns = float(row["AverageNs"])
                m = re.search(kpat + r"<[^>]*>", row["Name"])
                kname = m.group(0) if m else row["Name"][:60]
    fetch = np.median(counters(os.path.join(src, "fetch", "p_counter_collection.csv"), kpat)["FETCH_SIZE"])
    write = np.median(counters(os.path.join(src, "write", "p_counter_collection.csv"), kpat)["WRITE_SIZE"])
    cf = counters(os.path.join(src, "cfetch", "p_counter_collection.csv"), "calib")["FETCH_SIZE"]
    cw = counters(os.path.join(src, "cwrite", "p_counter_collection.csv"), "calib")["WRITE_SIZE"]
    # tools/calib_fetch.hip: 8 B/lane [T][K][2] (K 65536, T 64), or `4`: 4 B/lane [T][7][K] (K 131072, T 16)
    known_read, known_write = (58720256, 524288) if workload == "c5" else (33554432, 262144)
    f_ratio = np.median(cf) * 1024 / known_read
    w_ratio = np.median(cw) * 1024 / known_write
    read_b = fetch * 1024 / f_ratio
    write_b = write * 1024 / w_ratio
    alg = bps * K * T
    out = {
        "workload": workload, "K": K, "T": T, "kernel": kname + " (fused update)",
        "hbm_bytes_per_launch": int(round(read_b + write_b)),
        "read_bytes_per_launch": int(round(read_b)),
        "write_bytes_per_launch": int(round(write_b)),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "FETCH_SIZE_KB_median": fetch, "WRITE_SIZE_KB_median": write,
        "calibration": {"kernel": "tools/calib_fetch.hip " + ("4 (the chain's 4 B/lane [T][7][K] rows)" if workload == "c5"
                                                              else "(same 8 B/lane [T][K][2] row pattern)"),
                        "known_read_bytes": known_read, "FETCH_SIZE_KB": float(np.median(cf)),
                        "fetch_reported_over_true": f_ratio, "known_write_bytes": known_write,
                        "WRITE_SIZE_KB": float(np.median(cw)), "write_reported_over_true": w_ratio},
        "rocprof_avg_kernel_ns": avg_ns,
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py; {os.path.basename(dst)}",
    }
    sqf = os.path.join(src, "sq", "p_counter_collection.csv")
    sq = {k: float(np.median(v)) for k, v in counters(sqf, kpat).items()} if os.path.exists(sqf) else {}
    if "SQ_INSTS_VALU" in sq:
        # whole-device VALU wave-instructions per launch (bench.py's "valu" roofline)
        out["valu_insts_per_launch"] = sq["SQ_INSTS_VALU"]
        out["waves_per_launch"] = sq.get("SQ_WAVES")
        if "SQ_ACTIVE_INST_VALU" in sq and "SQ_WAVE_CYCLES" in sq:
            # both in quad-cycles: the share of a wave's lifetime its VALU is executing, and
            # the cycles one VALU instruction occupies it (4 = the wave64 issue cadence)
            out["valu_active_frac_of_wave_time"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
            out["cycles_per_valu_inst"] = 4.0 * sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_INSTS_VALU"]
    name = sys.argv[6] if len(sys.argv) > 6 else ("traffic.json" if workload == "c3" else f"traffic_{workload}.json")
    json.dump(out, open(os.path.join(os.path.dirname(dst.rstrip('/')), name), "w"), indent=1)
    if sq:
        gr = {}
        grf = os.path.join(src, "grbm", "p_counter_collection.csv")
        if os.path.exists(grf):
            gr = {k: float(np.median(v)) for k, v in counters(grf, kpat).items()}
        summ = {"SQ": sq, "GRBM": gr}
        if "SQ_WAVE_CYCLES" in sq:
            summ["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"]
            summ["active_inst_frac"] = sq.get("SQ_ACTIVE_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"]
        if "SQ_WAVES" in sq and "SQ_INSTS_VALU" in sq:
            summ["valu_insts_per_wave"] = sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"]
        json.dump(summ, open(os.path.join(dst, "sq_counters.json"), "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "traffic_over_algorithmic", "rocprof_avg_kernel_ns")}))


if __name__ == "__main__":
    main()
