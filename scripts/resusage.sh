#!/bin/bash
# Per-kernel VGPR / scratch / occupancy / LDS of engine.hip (compile-time remarks, CPU only).
F=$(python3 -c "from reporter_amd import build; print(' '.join(build._flags()))")
/opt/rocm/bin/hipcc $F -Rpass-analysis=kernel-resource-usage -c ${1:-reporter_amd/csrc/engine.hip} -o /tmp/_ru.o 2>&1 |
python3 -c "
import re,sys
cur=None
rows={}
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); rows[cur]={}; continue
    for k in ('VGPRs','AGPRs','ScratchSize \[bytes/lane\]','Occupancy \[waves/SIMD\]','LDS Size \[bytes/block\]','SGPRs'):
        m=re.search(k+r': (\d+)',l)
        if m and cur: rows[cur][k.split()[0]]=m.group(1)
for n,r in rows.items():
    if 'rocprim' in n: continue
    n=re.sub(r'_ZN2rm12_GLOBAL__N_1\d+','',n)[:40]
    print('%-40s vgpr=%-4s agpr=%-3s scratch=%-5s occ=%-3s lds=%s'%(n,r.get('VGPRs'),r.get('AGPRs'),r.get('ScratchSize'),r.get('Occupancy'),r.get('LDS')))
"
