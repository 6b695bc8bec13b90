"""Steady-state vmcnt simulation of a loop body in a gfx950 .s listing (diagnostic only).
usage: python3 tools/waitsim.py file.s first_line last_line
For every s_waitcnt vmcnt(N): how many loads it retires, how many chunk-compute lines ago the
youngest retired load was issued, and which register the following instructions read first."""
import re, sys
lines = open(sys.argv[1]).read().split("\n")[int(sys.argv[2]) - 1:int(sys.argv[3])]
def regs(s):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]|v(\d+)", s):
        if m.group(3): out.add(int(m.group(3)))
        else: out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out
fifo = []  # (line, dest regs)
for rep in range(3):
    for i, l in enumerate(lines):
        t = l.split(";")[0].strip()
        if not t or t.endswith(":"): continue
        op = t.split()[0]
        if op.startswith("global_load") or op.startswith("buffer_load"):
            dst = t.split()[1].rstrip(",")
            fifo.append((i, regs(dst)))
        elif op.startswith("global_store") or op.startswith("buffer_store"):
            fifo.append((i, set()))
        elif op == "s_waitcnt" and "vmcnt" in t:
            n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
            popped = []
            while len(fifo) > n: popped.append(fifo.pop(0))
            if rep == 2 and popped:
                pk_between = sum(1 for x in lines[popped[-1][0]:i] if "v_pk_" in x)
                nxt = next((x.strip() for x in lines[i + 1:i + 8] if x.strip().startswith("v_")), "")
                print("line %d: vmcnt(%d) retires %d, youngest retired issued %d lines / %d pk ops before; next: %s"
                      % (int(sys.argv[2]) + i, n, len(popped), i - popped[-1][0], pk_between, nxt[:60]))
