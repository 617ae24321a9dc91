"""Instruction mix of a kernel's ISA per s_memtime segment (stamp builds).

usage: python tools/isa_segs.py build/st_kernels.s <mangled-kernel-name> [seg-to-print]
"""
import collections
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
body = [l for l in s[i:j].split('\n')
        if l.strip() and not l.strip().startswith((';', '.'))]
seg, out = 0, {}
for l in body:
    if 's_memtime' in l:
        seg += 1
    out.setdefault(seg, []).append(l)


def kind(op):
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global', 'buffer', 'flat')):
        return 'vmem'
    return op


tot = collections.Counter()
for k, v in sorted(out.items()):
    c = collections.Counter(kind(l.split()[0]) for l in v)
    tot.update(c)
    print(k, len(v), dict(c))
print('total', sum(tot.values()), dict(tot))
if len(sys.argv) > 3:
    print('\n'.join(x[:100] for x in out[int(sys.argv[3])]))
