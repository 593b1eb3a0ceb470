"""Scan gfx950 device assembly (hipcc --cuda-device-only -S) for DPP instructions inside
inline asm whose DPP source VGPR was written by one of the two preceding VALU instructions
with no s_nop >= 1 in between: a VALU-write -> DPP-read hazard the compiler's hazard
recognizer does not see inside asm statements (it found the round-5 epilogue bug of
k_render_tile).  usage: dpp_hazard_scan.py file.s  (prints each hazard, then "hazards N")"""
import re
import sys
L=[l.strip() for l in open(sys.argv[1])]
fn=None; hist=[]; inasm=False; bad=0
def dst(l):
    op=l.split()[0]
    if op.startswith(('v_readlane','v_readfirstlane','v_cmp')): return None
    ops=l.split(None,1)
    if len(ops)<2: return None
    m=re.match(r'v\[?(\d+)', ops[1])
    return m.group(1) if m else None
for l in L:
    m=re.match(r'^(_Z\w+):',l)
    if m: fn=m.group(1); hist=[]; continue
    if ';;#ASMSTART' in l: inasm=True; continue
    if ';;#ASMEND' in l: inasm=False; continue
    if not l or l.startswith(';') or l.startswith('.'):
        if l.startswith('.LBB'): hist=[]
        continue
    op=l.split()[0]
    if op=='s_nop':
        n=int(l.split()[1]); hist = [] if n>=1 else [None]+hist[:1]; continue
    if op.startswith('v_') and '_dpp' in op and inasm:
        src=re.findall(r'v(\d+)', l.split(None,1)[1])[1]
        if src in hist[:2]: bad+=1; print(fn[:60], 'HAZARD', l)
    if op.startswith('v_'): hist=[dst(l)]+hist[:1]
    else: hist=[None]+hist[:1]
print('hazards', bad)
