"""Count instructions of named kernels in a gfx950 .s file (ISA probes).
Usage: python tools/experimental/isa_count.py FILE.s KERNEL [KERNEL ...]"""
import re,collections,sys
s=open(sys.argv[1]).read()
for name in sys.argv[2:]:
    m=re.search(r'\n'+name+r':[^\n]*\n(.*?)s_endpgm',s,re.S)
    body=m.group(1)
    ins=[l.strip().split()[0] for l in body.splitlines() if l.strip() and not l.strip().startswith(('.',';')) and not l.strip().endswith(':') and not l.strip().split()[0].endswith(':')]
    c=collections.Counter(ins)
    valu=sum(v for k,v in c.items() if k.startswith('v_'))
    print(name,'total',len(ins),'valu',valu,'mad',c['v_mad_u64_u32'])
    print('  ',c.most_common(16))
