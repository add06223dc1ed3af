#!/usr/bin/env python3
"""Summarise scripts/pmc_lds.sh output: per family case of k_pair_wave, the mean over
dispatches of LDS bank-conflict rate, LDS-stall share of CU time, occupancy and VALU
instructions per task.

Units (gfx950, 8 XCDs x 4 SEs, 256 CUs): SQ_BUSY_CYCLES is summed over the 32 SEs, so
/32 gives the kernel's cycles; SQ_WAVE_CYCLES counts quad-cycles summed over waves;
SQ_LDS_BANK_CONFLICT and SQ_LDS_IDX_ACTIVE are cycles summed over CUs.
"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_lds"
dst = sys.argv[2] if len(sys.argv) > 2 else None
N_TASKS = 65536  # every case has 65,536 keys per operand, all matched
out = {}
for f in sorted(glob.glob(os.path.join(src, "*", "run_counter_collection.csv"))):
    tag = f.split(os.sep)[-2]
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    name = {}
    for r in csv.DictReader(open(f)):
        d = r["Dispatch_Id"]
        disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name[d] = r["Kernel_Name"].split("(")[0]
    rows = []
    for d, c in disp.items():
        cyc = c["SQ_BUSY_CYCLES"] / 32
        rows.append({
            "kernel": name[d],
            "ms": dur[d],
            "lds_conflicts_per_access": c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_LDS_IDX_ACTIVE"] - c["SQ_LDS_BANK_CONFLICT"]),
            "lds_conflict_pct_of_cu_time": 100 * c["SQ_LDS_BANK_CONFLICT"] / (cyc * 256),
            "lds_active_pct_of_cu_time": 100 * c["SQ_LDS_IDX_ACTIVE"] / (cyc * 256),
            "lds_insts_per_task": c["SQ_INSTS_LDS"] / N_TASKS,
            "conflict_cycles_per_task": c["SQ_LDS_BANK_CONFLICT"] / N_TASKS,
            "waves_per_cu": 4 * c["SQ_WAVE_CYCLES"] / (cyc * 256),
            "occupancy_pct_of_16_resident": 100 * 4 * c["SQ_WAVE_CYCLES"] / (cyc * 256) / 16,
            "valu_insts_per_task": c["SQ_INSTS_VALU"] / N_TASKS,
            "valu_busy_pct": 100 * 4 * c["SQ_INSTS_VALU"] / (cyc * 1024),
        })
    m = {k: round(sum(r[k] for r in rows) / len(rows), 4) for k in rows[0] if k != "kernel"}
    m["kernel"] = rows[0]["kernel"]
    m["dispatches"] = len(rows)
    out[tag] = m
for k, v in out.items():
    print(f"{k:12s} ms={v['ms']:.3f} conf/acc={v['lds_conflicts_per_access']:.3f} conf%={v['lds_conflict_pct_of_cu_time']:.1f} "
          f"lds%={v['lds_active_pct_of_cu_time']:.1f} waves/CU={v['waves_per_cu']:.1f} valu/task={v['valu_insts_per_task']:.0f} "
          f"valu%={v['valu_busy_pct']:.0f}")
if dst:
    json.dump(out, open(dst, "w"), indent=1)
