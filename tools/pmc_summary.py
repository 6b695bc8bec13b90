"""Average rocprofv3 PMC counters per kernel from a counter_collection.csv."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if k.startswith(("__amd", "vectorized")):
        continue
    print(k, {c: round(sum(x) / len(x), 1) for c, x in sorted(v.items())})
