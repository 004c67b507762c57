"""Check the device assembly for the split append's hazard (sweep_sparse.hpp SP_SPLIT_APPEND).

sp_append_issue issues the wave's returning `global_atomic_add_x2` from inline asm, and
sp_append_finish waits for it with a manual `s_waitcnt vmcnt(0)` one loop iteration later.  The
compiler's wait-count pass does not see memory operations inside inline asm, so nothing but this
check guarantees that no instruction between the two reads (or overwrites) the atomic's destination
registers while the returned value is still in flight -- e.g. a copy of A.old_q the register
allocator might insert at the loop back-edge.

The check walks EVERY control-flow path from each such asm atomic (basic blocks split at labels and
branches of the .s listing) to the first `s_waitcnt` with vmcnt(0) on that path and fails if an
instruction on the way names one of the destination VGPRs.

    python tools/check_split_append.py sdfgenfast_amd/build/sdfgen_hip.s     (make -C sdfgenfast_amd asm)
Exit status 0 = safe; 1 = a hazard (printed); 2 = no split-append atomic found (the check is stale).
"""
import re
import sys

REG1 = re.compile(r"\bv(\d+)\b")
REGN = re.compile(r"\bv\[(\d+):(\d+)\]")
LABEL = re.compile(r"^([.\w$]+):")
BRANCH = re.compile(r"^\s*(s_branch|s_cbranch_\w+)\s+([.\w$]+)")


def regs_of(text):
    out = set(int(m) for m in REG1.findall(text))
    for a, b in REGN.findall(text):
        out.update(range(int(a), int(b) + 1))
    return out


def functions(lines):
    """(name, [(kind, text)]) per kernel: kind 'label' or 'insn' (comments stripped)."""
    funcs, cur, name, in_asm = [], None, None, False
    for raw in lines:
        line = raw.split(";")[0].rstrip() if not raw.lstrip().startswith(";;#ASM") else raw.strip()
        if raw.strip().startswith(";;#ASMSTART"):
            in_asm = True
            if cur is not None:
                cur.append(("asmstart", ""))
            continue
        if raw.strip().startswith(";;#ASMEND"):
            in_asm = False
            if cur is not None:
                cur.append(("asmend", ""))
            continue
        m = LABEL.match(line)
        if m:
            lab = m.group(1)
            if lab.startswith("_Z") and not lab.startswith(".L"):
                name, cur = lab, []
                funcs.append((name, cur))
            elif cur is not None:
                if lab.startswith(".Lfunc_end"):
                    cur = None
                else:
                    cur.append(("label", lab))
            continue
        if cur is None or not line.strip() or line.lstrip().startswith("."):
            continue
        cur.append(("insn", line.strip()))
    return funcs


def check_function(name, body):
    """Returns (n_atomics, [problems])."""
    labels = {t: i for i, (k, t) in enumerate(body) if k == "label"}
    problems, n = [], 0
    for i, (k, t) in enumerate(body):
        if k != "insn" or not t.startswith("global_atomic_add_x2") or " sc0" not in t:
            continue
        if not (i > 0 and body[i - 1][0] == "asmstart"):
            continue   # compiler-generated atomics are tracked by its own wait-count pass
        n += 1
        dst = regs_of(t.split(",")[0])
        # DFS over instruction indices after the asm block
        start = i + 1
        while start < len(body) and body[start][0] != "asmend":
            start += 1
        stack, seen = [start + 1], set()
        while stack:
            j = stack.pop()
            while j < len(body):
                if j in seen:
                    break
                seen.add(j)
                kind, text = body[j]
                if kind != "insn":
                    j += 1
                    continue
                if text.startswith("s_waitcnt") and "vmcnt(0)" in text:
                    break
                if text.startswith("s_endpgm"):
                    break
                hit = regs_of(text) & dst
                if hit:
                    problems.append(f"{name}: '{text}' names v{sorted(hit)} of in-flight '{t}' before s_waitcnt vmcnt(0)")
                bm = BRANCH.match(text)
                if bm:
                    tgt = labels.get(bm.group(2))
                    if tgt is None:
                        problems.append(f"{name}: branch to unknown label {bm.group(2)}")
                    else:
                        stack.append(tgt)
                    if bm.group(1) == "s_branch":
                        break
                if text.startswith(("s_setpc", "s_swappc")):
                    problems.append(f"{name}: indirect control flow '{text}' after the atomic")
                    break
                j += 1
    return n, problems


def main(path):
    with open(path) as f:
        lines = f.read().splitlines()
    total, probs = 0, []
    for name, body in functions(lines):
        n, p = check_function(name, body)
        total += n
        probs += p
        if n:
            print(f"{name}: {n} split-append atomic(s), every path waits before touching the result"
                  if not p else f"{name}: {len(p)} hazard(s)")
    for p in probs:
        print("HAZARD", p)
    if total == 0:
        print("no inline-asm returning global_atomic_add_x2 found: the check is stale")
        return 2
    return 1 if probs else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
