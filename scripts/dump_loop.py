"""Print the MFMA-carrying basic blocks of one kernel from a hipcc -S dump.
usage: dump_loop.py file.s substring-of-mangled-name"""
import re
import sys

s = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
start = [i for i, l in enumerate(s) if re.match(r'^[_A-Za-z][^\s]*:', l) and key in l.split(':')[0]][0]
end = [i for i in range(start, len(s)) if s[i].startswith('.Lfunc_end')][0]
body = s[start:end]
labels = [i for i, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)]
for li, l in enumerate(labels):
    nxt = labels[li + 1] if li + 1 < len(labels) else len(body)
    blk = [x for x in body[l:nxt] if x.strip() and not x.strip().startswith(';')]
    if any('mfma' in x for x in blk):
        print(body[l], len(blk), 'instrs')
        print('\n'.join(blk))
for l in s[end:end + 400]:
    if ('num_vgpr' in l or 'private_seg' in l or 'spill' in l) and key in l:
        print(l)
