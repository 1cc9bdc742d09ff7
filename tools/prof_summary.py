"""Summarise a tools/profile_round.sh run: rocprofv3 kernel stats + PMC FETCH_SIZE/WRITE_SIZE.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read stream, so reads are
doubled (the guide's calibration for 16-B-per-lane streaming), writes taken as reported.

  python tools/prof_summary.py gpurun_out/prof_r01 profiles/pmc_c3.json [--md profiles/x.md]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"bic(?:::|\d)([a-z_0-9]+?)(?:I|E|$)", name)
    if "k_" in name:
        m2 = re.search(r"(k_[a-z0-9_]+)", name)
        if m2:
            return m2.group(1)
    return m.group(1) if m else name[:40]


def load_counters(path):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[(short(row["Kernel_Name"]), row["Counter_Name"])].append(float(row["Counter_Value"]))
    return acc


def main():
    d, out = sys.argv[1], sys.argv[2]
    stats = {}
    with open(f"{d}/trace/run_kernel_stats.csv") as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            s = stats.setdefault(k, {"calls": 0, "total_ns": 0.0})
            s["calls"] += int(row["Calls"])
            s["total_ns"] += float(row["TotalDurationNs"])
    fetch = load_counters(f"{d}/fetch/run_counter_collection.csv")
    write = load_counters(f"{d}/write/run_counter_collection.csv")
    res = {"source": d, "method": "rocprofv3 --kernel-trace --stats; separate --pmc FETCH_SIZE / WRITE_SIZE passes; "
                                 "hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 read correction)",
           "kernels": {}}
    try:
        with open(f"{d}/sources.sha256") as f:
            res["sources_sha256"] = f.read().strip()
    except OSError:
        res["sources_sha256"] = None
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["total_ns"]):
        f = fetch.get((k, "FETCH_SIZE"), [])
        w = write.get((k, "WRITE_SIZE"), [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        hbm = (2 * fk * 1024 + wk * 1024) if (fk is not None and wk is not None) else None
        res["kernels"][k] = {"calls": s["calls"], "avg_us": round(s["total_ns"] / s["calls"] / 1e3, 2),
                             "fetch_kib": fk, "write_kib": wk,
                             "hbm_bytes_per_launch": int(hbm) if hbm is not None else None}
    # bench.py times launch sequences (bic_prof_* names); their HBM bytes per launch are the sums
    # over the kernels each sequence runs, per launch of its main kernel
    # (the first kernel of each list runs once per launch of the sequence: it gives the count)
    rows = ["k_emit_known", "k_emit_rest", "k_encode_rows", "k_len_rows", "k_emit_rows"]
    timers = {"encode_rows_golomb_eg": rows, "encode_rows_golomb": rows, "encode_rows_eg": rows,
              "encode_rows_golomb_egsrc": ["k_emit_k01", "k_emit_rest", "k_emit_known"],
              "encode_prefix": ["k_row_walk", "k_scan_rows", "k_med_kstat"],
              "bitplanes_count": ["k_gray_strips"],
              "encode_finish": ["k_rows_global", "k_fixup"],
              "bitplanes_u8": ["k_bitplanes_u8"], "med_count": ["k_med_rows", "k_count", "k_plane_weight"],
              "tiles": ["k_tiles_aligned", "k_tiles", "k_tiles_split"], "golomb_samples": ["k_samp_scan", "k_samp_emit"],
              "pack": ["k_pack"]}
    res["timers"] = {}
    K = res["kernels"]
    for t, ks in timers.items():
        present = [k for k in ks if k in K and K[k]["hbm_bytes_per_launch"] is not None]
        if not present:
            continue
        launches = K[present[0]]["calls"]
        tot = sum(K[k]["hbm_bytes_per_launch"] * K[k]["calls"] for k in present)
        res["timers"][t] = {"kernels": present, "launches": launches, "hbm_bytes_per_launch": int(tot / launches)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:28s} calls={v['calls']:4d} avg_us={v['avg_us']:10.2f} hbm_MB/launch="
              f"{(v['hbm_bytes_per_launch'] or 0) / 1e6:10.2f}")


if __name__ == "__main__":
    main()
