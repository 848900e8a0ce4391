"""Per-basic-block instruction mix of one kernel in a hipcc -S dump."""
import collections
import re
import sys

s = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
start = [i for i, l in enumerate(s) if re.match(r'^[_A-Za-z][^\s]*:', l) and key in l.split(':')[0]][0]
end = [i for i in range(start, len(s)) if s[i].startswith('.Lfunc_end')][0]
body = s[start:end]
labels = [0] + [i for i, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)]
tot = collections.Counter()
for li, l in enumerate(labels):
    nxt = labels[li + 1] if li + 1 < len(labels) else len(body)
    blk = [x.strip() for x in body[l:nxt][1:] if x.strip() and not x.strip().startswith((';', '.'))]
    c = collections.Counter()
    for x in blk:
        op = x.split()[0]
        k = ('mfma' if op.startswith('v_mfma') else 'valu' if op.startswith('v_') else
             'lds' if op.startswith('ds_') else
             'vmem' if op.startswith(('global_', 'buffer_')) else 'salu' if op.startswith('s_') else 'other')
        c[k] += 1
    tot += c
    if len(blk) >= int(sys.argv[3] if len(sys.argv) > 3 else 20):
        print(body[l].split(':')[0] if l else 'entry', len(blk), dict(c))
print('total', dict(tot))
for l in s[end:end + 600]:
    if key in l and ('num_vgpr' in l or 'private_seg_size' in l):
        print(l.strip())
