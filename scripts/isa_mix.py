#!/usr/bin/env python3
"""Instruction mix of a kernel's MFMA-heavy basic blocks in a gfx950 device .s file.
usage: isa_mix.py <file.s> <mangled-name-substring> [min_mfma]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
sub, min_mfma = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 12
m = re.search(r'^(_Z\S*' + re.escape(sub) + r'\S*):', s, re.M)
name = m.group(1)
body = s[m.end():]
body = body[:body.index('.Lfunc_end')]
blocks, cur = [], ['entry', []]
blocks.append(cur)
for l in body.split('\n'):
    l = l.strip()
    if re.match(r'^\.LBB\S+:', l):
        cur = [l, []]
        blocks.append(cur)
        continue
    if l and not l.startswith(('.', ';', '//')):
        cur[1].append(l.split()[0])
print(name)
for bname, ins in blocks:
    c = Counter(ins)
    mf = sum(v for k, v in c.items() if 'mfma' in k)
    if mf < min_mfma:
        continue
    valu = sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k)
    ds = sum(v for k, v in c.items() if k.startswith('ds_'))
    sm = sum(v for k, v in c.items() if k.startswith('s_'))
    gl = sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))
    print(f"{bname} instr {len(ins)} mfma {mf} valu {valu} ds {ds} salu {sm} global {gl}")
    print("   ", [(k, v) for k, v in c.most_common(60) if k.startswith('v_') and 'mfma' not in k][:30])
