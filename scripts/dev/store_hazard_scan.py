"""Dev: scan a kernel assembly (hipcc -S --cuda-device-only) for a 12/16-byte store followed, with no wait state,
by a VALU write of its data registers (the gfx950 hazard of DESIGN.md section 8, sampled modes).
usage: python scripts/dev/store_hazard_scan.py kernel.s"""
import re,sys
lines=open(sys.argv[1]).read().split('\n')
def regs(tok):
    m=re.match(r'v\[(\d+):(\d+)\]',tok)
    if m: return set(range(int(m.group(1)),int(m.group(2))+1))
    m=re.match(r'v(\d+)$',tok)
    return {int(m.group(1))} if m else set()
fn=None; cnt={}
for i,l in enumerate(lines):
    if re.match(r'^_Z\S*:',l): fn=l.split(':')[0][:60]
    m=re.match(r'\s+(buffer_store_dwordx[234]|global_store_dwordx[234]|buffer_store_dwordx2|scratch_store_dwordx[234])\s+(\S+?),\s*(\S+?),',l)
    if not m: continue
    op=m.group(1)
    data = regs(m.group(2)) if op.startswith('buffer') else regs(m.group(3)) if op.startswith('global') else regs(m.group(3))
    if op.startswith('scratch'): data=regs(m.group(3))
    # next non-comment instructions
    j=i+1; k=0
    while j<len(lines) and k<2:
        t=lines[j].strip()
        if not t or t.startswith(';') or t.endswith(':'): j+=1; continue
        if t.startswith('s_nop'): break
        parts=t.split(None,1)
        if len(parts)>1 and parts[0].startswith('v_'):
            dst=parts[1].split(',')[0].strip()
            if regs(dst)&data:
                print(fn, i+1, l.strip(), '||', t); cnt[fn]=cnt.get(fn,0)+1
        k+=1; j+=1
print(cnt)
