"""Per-dispatch averages of the pmc_fam.sh counters, per family pair."""
import collections, csv, glob, os, sys
base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_fam"
for d in sorted(glob.glob(base + "/*/")):
    rows = list(csv.DictReader(open(glob.glob(d + "*counter_collection.csv")[0])))
    per = collections.defaultdict(dict)
    for r in rows:
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    last = per[sorted(per, key=int)[-1]]
    tasks = 65536
    wc = last["SQ_WAVE_CYCLES"]
    print(os.path.basename(d.rstrip("/")), "VALU/task %.0f LDS/task %.0f" % (last["SQ_INSTS_VALU"] / tasks, last["SQ_INSTS_LDS"] / tasks),
          "active %.2f wait %.2f waitinst %.2f" % (last["SQ_ACTIVE_INST_ANY"] / wc, last["SQ_WAIT_ANY"] / wc, last["SQ_WAIT_INST_ANY"] / wc),
          "VALU-cycles/SIMD %.0f" % (last["SQ_INSTS_VALU"] * 4 / 1024))
