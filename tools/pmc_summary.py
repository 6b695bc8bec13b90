"""Per-kernel rocprofv3 PMC counters from a counter_collection.csv: each counter summed over its
instances (XCDs / shader engines) per dispatch, then averaged over the kernel's dispatches.
Kernels are keyed by name including template arguments (e.g. the decoder's MODE)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = collections.defaultdict(float)
names = {}
for r in rows:
    key = (r["Dispatch_Id"], r["Counter_Name"])
    per[key] += float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for (disp, ctr), v in per.items():
    acc[names[disp][:72]][ctr].append(v)
for k, v in sorted(acc.items()):
    if k.startswith(("__amd", "vectorized")):
        continue
    print(k, {c: round(sum(x) / len(x), 1) for c, x in sorted(v.items())})
