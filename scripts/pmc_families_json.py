#!/usr/bin/env python3
"""profiles/<round>/pmc_families.json from scripts/pmc_attrib.sh output.

Per family case of k_pair_wave (65,536 tasks): LDS bank-conflict cycles per LDS instruction and
their share of CU time, achieved occupancy (waves per SIMD against the launch bound of 4: 4
workgroups x 4 waves per CU), VALU per task -- from the default library ("base") -- and the
conflict cycles attributed to named accesses by the attribution builds: "probelin" makes the
filter's map probes lane-linear (conflict-free) and "scatlin" the array scatter's LDS atomics;
the conflict cycles each removes are that access's share, the rest is the other LDS traffic
(run toggles and prefix pass, staging of array / run results, compaction, row reductions).

usage: pmc_families_json.py gpurun_out profiles/r04/pmc_families.json
"""
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]


def load(v):
    p = os.path.join(src, f"pmc_lds_{v}.json")
    return json.load(open(p)) if os.path.exists(p) else {}


base, plin, slin = load("base"), load("probelin"), load("scatlin")
out = {"_units": {
    "conflict_cycles_per_lds_inst": "SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (all LDS instructions of the kernel)",
    "lds_conflict_pct_of_cu_time": "SQ_LDS_BANK_CONFLICT / (kernel cycles x 256 CUs)",
    "waves_per_simd": "SQ_WAVE_CYCLES x 4 / (kernel cycles x 256 CUs) / 4 SIMDs; launch bound 4",
    "attribution": "conflict cycles per task removed by the lane-linear probe / scatter builds (timing-only)"}}
for tag, b in base.items():
    insts = b["lds_insts_per_task"]
    row = {
        "ms": b["ms"],
        "lds_insts_per_task": round(insts, 1),
        "lds_conflict_pct_of_cu_time": b["lds_conflict_pct_of_cu_time"],
        "lds_active_pct_of_cu_time": b["lds_active_pct_of_cu_time"],
        "lds_conflicts_per_access": b["lds_conflicts_per_access"],
        "waves_per_cu": b["waves_per_cu"],
        "waves_per_simd": round(b["waves_per_cu"] / 4, 2),
        "launch_bound_waves_per_simd": 4,
        "valu_insts_per_task": b["valu_insts_per_task"],
        "valu_busy_pct": b["valu_busy_pct"],
    }
    if "conflict_cycles_per_task" in b:
        row["conflict_cycles_per_task"] = b["conflict_cycles_per_task"]
        row["conflict_cycles_per_lds_inst"] = round(b["conflict_cycles_per_task"] / max(insts, 1e-9), 3)
        attr = {}
        for name, d in (("map_probe", plin), ("array_scatter", slin)):
            if tag in d and "conflict_cycles_per_task" in d[tag]:
                attr[name] = round(b["conflict_cycles_per_task"] - d[tag]["conflict_cycles_per_task"], 1)
                attr[name + "_ms_timing_only"] = d[tag]["ms"]
        if attr:
            attr["other"] = round(b["conflict_cycles_per_task"] - attr.get("map_probe", 0) - attr.get("array_scatter", 0),
                                  1)
            row["attribution_conflict_cycles_per_task"] = attr
    out[tag] = row
json.dump(out, open(dst, "w"), indent=1)
for k, v in out.items():
    if k.startswith("_"):
        continue
    print(k, v.get("conflict_cycles_per_lds_inst"), v["waves_per_simd"], v.get("attribution_conflict_cycles_per_task"))
