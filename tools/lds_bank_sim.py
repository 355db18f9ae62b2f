import collections
def mc_swz(CH,k): return ((((k & 3) | (((k >> 3) & 1) << 2)) << 1) & (CH - 1))
def groups(kind):
    if kind in ('b64','tr'): return [list(range(0,32)), list(range(32,64))]
    if kind=='b128': return [[0,1,2,3,12,13,14,15]+list(range(20,28)), list(range(4,12))+[16,17,18,19]+list(range(28,32)), [32,33,34,35,44,45,46,47]+list(range(52,60)), list(range(36,44))+[48,49,50,51]+list(range(60,64))]
    if kind=='w64': return [list(range(i,i+16)) for i in range(0,64,16)]
def cost(addrs, nbytes, kind):
    nb = 32 if kind=='w64' else 64
    tot=0
    for g in groups(kind):
        banks=collections.defaultdict(set)
        for l in g:
            a=addrs[l]
            for d in range(nbytes//4):
                dw=a//4+d
                banks[dw%nb].add(dw)
        tot+=max(len(v) for v in banks.values())
    return tot, len(groups(kind))
def frag_mc(ROWS, r0, ks):
    CH=ROWS//8; A=[];B=[]
    for lane in range(64):
        g=lane>>4; i=lane&15; q=i>>2; p=i&3
        kA=ks*32+8*g+q; kB=kA+4; ch=(r0>>3)+(p>>1); sub=(p&1)*8
        A.append(kA*ROWS*2+((ch^mc_swz(CH,kA))<<4)+sub); B.append(kB*ROWS*2+((ch^mc_swz(CH,kB))<<4)+sub)
    return A,B
def kc_off(row,k): return row*128+((((k>>3)^(row&7)))<<4)+(k&7)*2
def frag_kc(r0,ks):
    return [ (r0+(l&15))*128 + ((((ks*4+(l>>4)) ^ ((r0+(l&15))&7)))<<4) for l in range(64)]
print("fwd V frag_mc<64> tr reads:")
for j in range(4):
    for ks in range(2):
        A,B=frag_mc(64,j*16,ks); print(" j",j,"ks",ks, cost(A,8,'tr'), cost(B,8,'tr'))
print("fwd P st4 (ds_write_b64):")
for j in range(4):
    ad=[kc_off(l&15, j*16+4*(l>>4)) for l in range(64)]
    print(" j",j,cost(ad,8,'w64'))
print("fwd P frag_kc reads:", [cost(frag_kc(0,ks),16,'b128') for ks in range(2)])
print("fwd K frag_kc reads:", [cost(frag_kc(j*16,ks),16,'b128') for j in range(4) for ks in range(2)])
# final O store: scr + qi*128 + (j*16+4g)*2, 8 bytes
print("fwd O st4:", [cost([ (l&15)*128 + (j*16+4*(l>>4))*2 for l in range(64)],8,'w64') for j in range(4)])
print("=== new swizzle for CH=8")
def mc_swz_new(CH,k):
    if CH==8: return (((k & 3) << 1) | ((k >> 3) & 1)) & 7
    return mc_swz(CH,k)
def frag_mc_sw(ROWS, r0, ks, sw):
    CH=ROWS//8; A=[];B=[]
    for lane in range(64):
        g=lane>>4; i=lane&15; q=i>>2; p=i&3
        kA=ks*32+8*g+q; kB=kA+4; ch=(r0>>3)+(p>>1); sub=(p&1)*8
        A.append(kA*ROWS*2+((ch^sw(CH,kA))<<4)+sub); B.append(kB*ROWS*2+((ch^sw(CH,kB))<<4)+sub)
    return A,B
for name,sw in (("old",mc_swz),("new",mc_swz_new)):
    res=[]
    for r0 in (0,16,32,48):
        for ks in (0,1):
            A,B=frag_mc_sw(64,r0,ks,sw); res.append((cost(A,8,'tr')[0],cost(B,8,'tr')[0]))
    print(name,"frag_mc<64>",res)
    # bwd Q/dO row reads (ds_read_b128): qrow = base + (lane&15), cb = lane>>4, chunks cb^sw and (4+cb)^sw
    res=[]
    for base in (0,16,32,48):
        for hi in (0,4):
            ad=[ (base+(l&15))*128 + ((((hi+(l>>4)) ^ sw(8, base+(l&15))))<<4) for l in range(64)]
            res.append(cost(ad,16,'b128')[0])
    print(name,"bwd Q/dO row reads (ideal 4)",res)
    # 128-row MC (CH=16) check unchanged
    A,B=frag_mc_sw(128,0,0,sw); print(name,"frag_mc<128>",cost(A,8,'tr'),cost(B,8,'tr'))
print("=== candidate swizzle")
def mc_swz_c(CH,k):
    if CH==8: return ((((k >> 3) & 1) << 2) | (((k >> 1) & 1) << 1) | (k & 1))
    return mc_swz(CH,k)
res=[]
for r0 in (0,16,32,48):
    for ks in (0,1):
        A,B=frag_mc_sw(64,r0,ks,mc_swz_c); res.append((cost(A,8,'tr')[0],cost(B,8,'tr')[0]))
print("cand frag_mc<64> (ideal 2)",res)
res=[]
for base in (0,16,32,48):
    for hi in (0,4):
        ad=[ (base+(l&15))*128 + ((((hi+(l>>4)) ^ mc_swz_c(8, base+(l&15))))<<4) for l in range(64)]
        res.append(cost(ad,16,'b128')[0])
print("cand bwd Q/dO row reads (ideal 4)",res)
