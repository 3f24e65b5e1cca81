"""Bank-conflict model of the fp16 MLP kernel's activation planes (MI355X_MICROARCH.md LDS table): ds_read_b128
B-fragment reads (lane groups {0-3,12-15,20-27}, ..., banks mod 64) and the epilogue's ds_write_b64 (16 contiguous
lanes, banks mod 32), over row strides and row swizzles of the 16-byte units; prints the worst N-way per pattern.

    python tools/lds_swizzle_search.py"""
import itertools
RG=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
RG=RG+[[x+32 for x in g] for g in RG]
def read_conf(RS, f, kc):
    worst=0
    for g in RG:
        banks={}
        for l in g:
            row, q = l & 15, l >> 4
            c = kc*4 + q
            a = row*RS + 16*(c ^ f(row))
            for d in range(4):
                b=(a//4 + d) % 64
                banks.setdefault(b,set()).add(a)
        worst=max(worst, max(len(v) for v in banks.values()))
    return worst
def write_conf(RS, f, nt):
    worst=0
    for G in range(4):
        banks={}
        for l in range(16*G, 16*G+16):
            row, q = l & 15, l >> 4
            chunk = 2*nt + (q >> 1); half = q & 1
            a = row*RS + 16*(chunk ^ f(row)) + 8*half
            for d in range(2):
                b=(a//4 + d) % 32
                banks.setdefault(b,set()).add(a)
        worst=max(worst, max(len(v) for v in banks.values()))
    return worst
fams = {
 'none': lambda r: 0,
}
for a in range(0,4):
    for m in (1,3,7):
        fams[f'(r>>{a})&{m}'] = (lambda a,m: (lambda r: (r>>a)&m))(a,m)
for mul in (1,2,3,5):
    for m in (3,7):
        fams[f'(r*{mul}>>2)&{m}'] = (lambda mul,m: (lambda r: ((r*mul)>>2)&m))(mul,m)
res=[]
for RS in range(256, 400, 16):
    for name,f in fams.items():
        rc=max(read_conf(RS,f,kc) for kc in range(4))
        wc=max(write_conf(RS,f,nt) for nt in range(8))
        res.append((rc+wc, rc, wc, RS, name))
res.sort()
for r in res[:15]: print(r)
print('current RS=288 none:', [r for r in res if r[3]==288 and r[4]=='none'])
f=lambda r: (r>>2)&1
for RS in (288, 544):
    print(RS, 'reads', max(read_conf(RS,f,kc) for kc in range(8)), 'writes', max(write_conf(RS,f,nt) for nt in range(16)),
          'no-swizzle reads', max(read_conf(RS,lambda r:0,kc) for kc in range(8)), 'writes', max(write_conf(RS,lambda r:0,nt) for nt in range(16)))
