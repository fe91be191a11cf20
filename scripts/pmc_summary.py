"""Summarise rocprofv3 --pmc passes: per miclip kernel name, counter averages over dispatches."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "miclip" not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"], r["Kernel_Name"].split("(")[0].replace("void miclip::(anonymous namespace)::", ""),
               r["Grid_Size"])
        per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for (d, name, grid), cs in per.items():
        for c, v in cs.items():
            acc[(name, grid)][c].append(v)
for (name, grid), cs in acc.items():
    print(f"== {name} grid={grid}")
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} {sum(vs) / len(vs):14.4g}  (n={len(vs)})")
