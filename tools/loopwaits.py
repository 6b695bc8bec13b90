"""For every loop of a gfx950 .s kernel listing with > 100 packed ops: the vmcnt waits of its
steady state (diagnostic only; tools/waitsim.py does the simulation)."""
import re, subprocess, sys
f = sys.argv[1]
L = open(f).read().split("\n")
labels = {}
for i, l in enumerate(L):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m: labels[m.group(1)] = i
for name, i0 in sorted(labels.items(), key=lambda x: x[1]):
    if "Loop Header" not in L[i0] and "Loop Header" not in L[i0 + 1]: continue
    ends = [j for j, l in enumerate(L) if re.search(r"s_c?branch\w* " + re.escape(name) + r"$", l) and j > i0]
    if not ends: continue
    i1 = max(ends)
    pk = sum(1 for l in L[i0:i1] if "v_pk_" in l)
    if pk < 100: continue
    ds = sum(1 for l in L[i0:i1] if "ds_" in l)
    print("== %s lines %d-%d pk %d ds %d" % (name, i0 + 1, i1 + 1, pk, ds))
    sys.stdout.flush()
    subprocess.run(["python3", "/root/repo/tools/waitsim.py", f, str(i0 + 1), str(i1 + 1)])
