"""Instruction-class counts per basic block (blocks over a size threshold) of one kernel in a
hipcc -S listing.  Tuning aid.  usage: python scripts/asmblocks.py file.s kernel_substring [min]"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    L = open(path).read().split('\n')
    st = [i for i, l in enumerate(L) if re.match(r'^_Z\S*' + re.escape(name) + r'\S*:', l)][0]
    en = [i for i in range(st, len(L)) if L[i].startswith('.Lfunc_end')][0]
    blocks, cur = [], None
    for i in range(st, en):
        m = re.match(r'^(\.LBB\w+):', L[i])
        if m:
            cur = [m.group(1), i + 1, collections.Counter(), 0]
            blocks.append(cur)
            continue
        t = L[i].strip()
        if cur is None or not t or t.startswith((';', '.')):
            continue
        op = t.split()[0]
        cur[3] += 1
        cls = ('mfma' if 'mfma' in op else 'exp' if op.startswith('v_exp') else 'valu' if op.startswith('v_') else
               'ds' if op.startswith('ds_') else 'vmem' if op.startswith(('global_', 'buffer_')) else
               'salu' if op.startswith('s_') else 'other')
        cur[2][cls] += 1
    for b in blocks:
        if b[3] >= lim:
            print(b[0], 'line', b[1], b[3], dict(b[2]))
    print([l for l in L if re.search(re.escape(name) + r'\S*\.num_vgpr', l)][:1])


if __name__ == '__main__':
    main()
