"""Condense variant_kinds.sh output (.and / .or compute phase ms per variant)."""
import re, sys
txt = open(sys.argv[1]).read()
for blk in txt.split("== ")[1:]:
    name = blk.split()[0]
    items = re.findall(r"(\S+) \[([^\]]*)\]", blk[len(name):])
    print(name, " ".join(f"{k}={v.split(',')[1].strip()}" for k, v in items if k.endswith(".and") or k.endswith(".or")))
