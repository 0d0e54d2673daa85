"""Bank-conflict simulation of k_conv_x9's A-fragment reads (ds_read_b128 lane groups of
MI355X_MICROARCH.md §LDS: four 16-lane groups, bank = (a/4) % 64): average LDS cycles per lane
group over every (tile, chunk) step of conv2 / conv3 at each built samples-per-workgroup, for
the kernel's rotation swizzle and an exhaustive search over rotations, shifts and plane pads.
Development aid (CPU only)."""
import itertools
GROUPS=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
GROUPS += [[l+32 for l in g] for g in GROUPS]
def geom(KH,KW,S,CIN,HIN,WIN,NSAMP):
    HOUT=(HIN-KH)//S+1; WOUT=(WIN-KW)//S+1; PIX=HOUT*WOUT; K=KH*KW*CIN; NCH=K//32
    TILES=(NSAMP*PIX+15)//16; NG=CIN//8; ROWS=NSAMP*HIN*WIN
    return dict(HOUT=HOUT,WOUT=WOUT,PIX=PIX,NCH=NCH,TILES=TILES,NG=NG,ROWS=ROWS)
def sim(KH,KW,S,CIN,HIN,WIN,NSAMP,swz,pad):
    G=geom(KH,KW,S,CIN,HIN,WIN,NSAMP)
    PLANE=(G['ROWS']+15)//16*16+pad
    nv=NSAMP*G['PIX']
    tot=0;cnt=0
    for c in range(G['NCH']):
        k0=c*32; tap=k0//CIN; toff=(tap//KW)*WIN+tap%KW; coff=((k0%CIN)//8)*PLANE
        for tile in range(G['TILES']):
            units=[]
            for l in range(64):
                p=tile*16+(l&15)
                if p>=nv: p=nv-1
                s=p//G['PIX']; pp=p-s*G['PIX']; oy=pp//G['WOUT']; ox=pp-oy*G['WOUT']
                r=s*HIN*WIN+S*oy*WIN+S*ox
                units.append(coff+(l>>4)*PLANE+swz(r+toff))
            for g in GROUPS:
                slots={}
                for l in g: slots.setdefault(units[l]%16,set()).add(units[l])
                tot+=max(len(v) for v in slots.values()); cnt+=1
    return tot/cnt
def mk(ROT,SH=5):
    # SH >= 4: the rotation is constant over each aligned 16-row block, so the map permutes it
    # (SH < 4 maps two rows of a block to one unit: not a valid swizzle -- X9Geom asserts it)
    assert SH >= 4
    return lambda r:(r&~15)|((r+(r>>SH)*ROT)&15)
def sim_tmap(KH, KW, S, CIN, HIN, WIN, NSAMP):
    """the tile map of k_conv_x9 (ROT < 0, stride 1): unit(s, y, x) = s SU + 16 y + ((WOUT y + x) mod 16),
    PLANE a multiple of 16, lanes past the last valid pixel read the pixel 16 before"""
    G = geom(KH, KW, S, CIN, HIN, WIN, NSAMP)
    SU = 16 * HIN + ((G['PIX'] - 16 * HIN) % 16)
    PLANE = (NSAMP * SU + 15) // 16 * 16
    nv = NSAMP * G['PIX']
    tot = cnt = 0
    for c in range(G['NCH']):
        k0 = c * 32; tap = k0 // CIN; dy, dx = tap // KW, tap % KW; coff = ((k0 % CIN) // 8) * PLANE
        for tile in range(G['TILES']):
            units = []
            for l in range(64):
                p = tile * 16 + (l & 15)
                p = p - 16 if p >= nv else p
                s, pp = divmod(p, G['PIX']); oy, ox = divmod(pp, G['WOUT'])
                y, x = oy + dy, ox + dx
                units.append(coff + (l >> 4) * PLANE + s * SU + 16 * y + ((G['WOUT'] * y + x) & 15))
            for g in GROUPS:
                slots = {}
                for l in g: slots.setdefault(units[l] % 16, set()).add(units[l])
                tot += max(len(v) for v in slots.values()); cnt += 1
    return tot / cnt, 3 * G['NG'] * PLANE * 16


for ns in (1, 2):
    c, lds = sim_tmap(3, 3, 1, 64, 9, 9, ns)
    print('conv3', ns, 'tile map %.2f cycles per group, %d KB of LDS' % (c, lds // 1024))
for name,geo,ns_list,cur in (("conv3",(3,3,1,64,9,9),(1,2,3,4),(3,0)),("conv2",(4,4,2,32,20,20),(1,2),(10,1))):
    for ns in ns_list:
        c=sim(*geo,ns,mk(cur[0]),cur[1])
        best=min(((sim(*geo,ns,mk(rot,sh),pad),rot,sh,pad) for rot in range(16) for sh in (4,5,6) for pad in (0,1,2,4,8)),key=lambda t:t[0])
        print(name,ns,'current %.2f'%c,'best %.2f rot %d sh %d pad %d'%best, 'identity %.2f'%sim(*geo,ns,lambda r:r,0))
