"""Where do a kernel's scratch (spill) instructions sit? Per basic block of each
kernel in a gfx950 .s file: VALU count, scratch op count, and whether the block
is a loop body (has a backward branch to itself). usage: spill_map.py file.s [substr]"""
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else "kernel"
for m in re.finditer(r"^(_Z\S*):[^\n]*\n(.*?)\.Lfunc_end", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if sub not in name:
        continue
    blocks = re.split(r'\n(?=\.LBB\S+:)', body)
    print(name)
    tot_sc = 0
    for b in blocks:
        lines = b.split('\n')
        lab = lines[0].rstrip(':') if lines[0].startswith('.LBB') else '(entry)'
        nsc = sum(1 for l in lines if 'scratch_' in l)
        nv = sum(1 for l in lines if re.match(r'\s+v_', l))
        loop = any(re.search(r's_cbranch\S*\s+' + re.escape(lab) + r'\b', l) or re.search(r's_branch\s+' + re.escape(lab) + r'\b', l) for l in lines)
        tot_sc += nsc
        if nsc:
            print(f'   {lab:18s} valu {nv:5d} scratch {nsc:4d} {"LOOP" if loop else ""}')
    print('   total scratch ops', tot_sc)
