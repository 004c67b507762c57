"""Loops of one kernel in an llvm-objdump listing (tools/kres.py's code object): instruction mix per
backward branch, innermost first -- where a step's instructions go.
    python tools/isa_loops.py LISTING.s KERNEL-SUBSTRING"""
import re
import sys

txt = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
start = next(i for i, l in enumerate(txt) if l.endswith(">:") and key in l)
end = next((i for i in range(start + 1, len(txt)) if txt[i].endswith(">:")), len(txt))
ins = []
for l in txt[start + 1:end]:
    m = re.match(r"\s+(\S+)\s.*//\s+([0-9A-F]+):", l)
    if m:
        ins.append((int(m.group(2), 16), m.group(1), l))
base = ins[0][0]
pos = {a: k for k, (a, _, _) in enumerate(ins)}
print(f"{len(ins)} instructions")
for k, (a, op, l) in enumerate(ins):
    if op.startswith("s_cbranch") or op == "s_branch":
        m = re.search(r"\+0x([0-9a-f]+)>", l)
        if not m:
            continue
        t = int(m.group(1), 16) + base
        if t <= a and t in pos:
            body = ins[pos[t]:k + 1]
            cnt = lambda p: sum(1 for x in body if x[1].startswith(p))
            print(f"  loop [{pos[t]}, {k}] {len(body):5d} instrs: v {cnt('v_'):4d} s {cnt('s_'):4d} ds {cnt('ds_'):3d} "
                  f"vmem {cnt('global_') + cnt('buffer_') + cnt('scratch_'):3d} dpp {sum(1 for x in body if 'dpp' in x[2] or 'quad_perm' in x[2] or 'row_' in x[2]):3d} ({op})")
