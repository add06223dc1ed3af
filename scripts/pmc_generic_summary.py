#!/usr/bin/env python3
"""Mean counter values per case directory of a rocprofv3 --pmc run tree:
   scripts/pmc_generic_summary.py gpurun_out/pmc_mem profiles/r01/pmc_memory.json
Case directories named TAG or TAG_gN (counter groups of one case) are merged."""
import collections
import csv
import glob
import json
import os
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(src, "*", "run_counter_collection.csv"))):
    tag = re.sub(r"_g\d+$", "", f.split(os.sep)[-2])
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        res[tag]["kernel"] = r["Kernel_Name"].split("(")[0]
    vals = collections.defaultdict(list)
    for c in disp.values():
        for k, v in c.items():
            vals[k].append(v)
    for k, v in vals.items():
        res[tag][k] = round(sum(v) / len(v), 1)
json.dump(res, open(dst, "w"), indent=1, sort_keys=True)
print(dst, list(res))
