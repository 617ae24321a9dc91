"""Static instruction mix of one kernel's loops, from the device assembly
(`make -C gym-simpletetris_amd/csrc asm` -> build/st_kernels.s).

For the kernel whose mangled name contains every given substring, prints
each loop (a backward branch to an earlier label) with the static count of
VALU / SALU / LDS / vector-memory / scalar-memory / branch / wait
instructions between its head label and its back edge (nested loops are
counted inside their parents too), and the kernel totals.  Static counts:
straight-line code is what a wave issues once per iteration; branches that
skip blocks make the dynamic count smaller.

usage: python tools/isa_loops.py build/st_kernels.s k_rollout Li10ELi20ELb0ELb1ELb0E
"""
import re
import sys


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_waitcnt") or op in ("s_barrier", "s_sleep", "s_setprio", "s_nop"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):", ln)
        if m and all(s in m.group(1) for s in subs):
            start = i
            name = m.group(1)
            break
    if start is None:
        sys.exit("kernel not found")
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start + 1:end]
    labels = {}
    ins = []  # (line index in body, op, text)
    for i, ln in enumerate(body):
        s = ln.strip()
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        ins.append((i, op, s))
    loops = []
    for k, (_, op, s) in enumerate(ins):
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= k:
                loops.append((labels[tgt], k, tgt))

    def mix(a, b):
        c = {}
        for _, op, _s in ins[a:b + 1]:
            k = classify(op)
            if k:
                c[k] = c.get(k, 0) + 1
        return c

    tot = mix(0, len(ins) - 1)
    print(f"{name}: {len(ins)} instructions  " + "  ".join(f"{k} {v}" for k, v in sorted(tot.items())))
    for a, b, tgt in sorted(loops):
        c = mix(a, b)
        print(f"  loop {tgt:14s} [{a:5d}, {b:5d}] {b - a + 1:5d} instr  " + "  ".join(f"{k} {v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
