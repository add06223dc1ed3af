#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/.

Writes
  profiles/<tag>/kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>/kernel_stats_<w>.csv  the same for workload w run alone (bench.py --only w)
  profiles/<tag>/bench_kt.json      the bench line printed under the kernel trace
  profiles/<tag>/pmc_summary.json   per-kernel mean counters over the --pmc passes
  profiles/pmc_traffic.json         HBM bytes per launch of each workload's dominant kernel, from
                                    that workload's own passes (read by bench.py)

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of 16 B/lane streaming reads, so it is
doubled; WRITE_SIZE is exact for 16 B/lane stores.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = "k_pair_cu<0, 0>"  # AND, results materialised (the bench headline kernel)


def short_name(n):
    """'void rbg::k_pair_wave<0, 0>(rbg::PTask const*, ...)' -> 'k_pair_wave<0, 0>'"""
    n = n.strip()
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):  # cut at the argument list (the first '(' outside <>)
        depth += ch == "<"
        depth -= ch == ">"
        if ch == "(" and depth == 0:
            n = n[:i]
            break
    return n.replace("rbg::", "").strip()


def kernel_stats(src, dst):
    """run_kernel_stats.csv with short names (template arguments kept)."""
    with open(src) as f:
        rows = list(csv.DictReader(f))
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()), quoting=csv.QUOTE_NONNUMERIC)
        w.writeheader()
        for r in rows:
            r["Name"] = short_name(r["Name"])
            w.writerow(r)


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return acc
    with open(path) as f:
        for row in csv.DictReader(f):
            name = short_name(row["Kernel_Name"])
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


# workload (bench.py --only) -> (traffic key in pmc_traffic.json, dominant kernel)
# (round 5: the dense pairwise ranges run the balanced list on one 16-wave workgroup per CU, k_pair_cu<OP, MODE>;
# round 6: k_serialize_agg is the whole placement + serialization of a pairwise result)
WORKLOADS = {"c2": ("k_pair_wave", "k_pair_cu<0, 0>"), "c2card": ("k_pair_wave_card", "k_pair_cu<0, 1>"),
             "c2ser": ("k_serialize_c2", "k_serialize_agg"), "c4": ("k_pair_items", "k_pair_items"),
             "c3u": ("k_wide<OR>_uniform", "k_wide<0>"), "c3c": ("k_wide<OR>_clustered", "k_wide<0>"),
             "c5": ("k_bsi_reg", "k_bsi_reg")}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    kt = os.path.join(src, "kt", "run_kernel_stats.csv")
    if os.path.exists(kt):
        kernel_stats(kt, os.path.join(dst, "kernel_stats.csv"))
    for w in [x for x in WORKLOADS if x != "c2ser"]:  # per-workload kernel traces (bench.py --only w)
        p = os.path.join(src, f"ktw_{w}", "run_kernel_stats.csv")
        if os.path.exists(p):
            kernel_stats(p, os.path.join(dst, f"kernel_stats_{w}.csv"))
    if os.path.exists(os.path.join(src, "bench_kt.json")):
        shutil.copy(os.path.join(src, "bench_kt.json"), os.path.join(dst, "bench_kt.json"))
    summary = {}
    for sub in sorted(os.listdir(src)):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not (sub.startswith("pmc_") or sub.startswith("sq_")) or not os.path.exists(p):
            continue
        w = sub.split("_")[1]
        for k, cs in counters(p).items():
            for c, vals in cs.items():
                summary.setdefault(w, {}).setdefault(k, {})[c] = {"mean": sum(vals) / len(vals), "n": len(vals)}
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    traffic = json.load(open(tp)) if os.path.exists(tp) else {}
    for w, (key, kern) in WORKLOADS.items():
        d = summary.get(w if w != "c2ser" else "c2", {}).get(kern, {})
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            rd = 2.0 * d["FETCH_SIZE"]["mean"] * 1024
            wr = d["WRITE_SIZE"]["mean"] * 1024
            traffic[key] = {"kernel": kern, "workload": w, "hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd),
                            "write_bytes": int(wr), "launches": d["FETCH_SIZE"]["n"],
                            "source": f"profiles/{tag}/pmc_summary.json ({w}, run alone)",
                            "correction": "FETCH_SIZE x2 (gfx950 streaming-read tally), KiB -> bytes"}
    with open(tp, "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
