import numpy as np
LAYS=[[6,7,8,0,1,2,3,4,5],[3,4,5,0,1,2,6,7,8],[0,1,2,4,5,8,3,6,7]]
def jof(li,lane,u):
    j=0
    for b in range(3): j|=((u>>b)&1)<<LAYS[li][b]
    for b in range(6): j|=((lane>>b)&1)<<LAYS[li][3+b]
    return j
def br9(j): return int(f"{j:09b}"[::-1],2)
E=np.array([[ (4*br9(jof(2,l,u))+1)&2047 for l in range(64)] for u in range(8)])
groups=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
groups+= [[g+32 for g in groups[0]],[g+32 for g in groups[1]]]
def cycles(pos):
    tot=0; worst=0
    for a in range(2048):
        for u in range(8):
            x=(a*E[u])&2047
            p=pos(x)
            c=0
            for g in groups:
                addrs=set(p[g].tolist())
                quads={}
                for ad in addrs: quads[ad%16]=quads.get(ad%16,0)+1
                c+=max(quads.values())
            tot+=c; worst=max(worst,c)
    return tot/(2048*8), worst
#print('plain', cycles(lambda x:x))
#print('xor4', cycles(lambda x: x ^ ((x>>4)&15)))
#print('xor4+8', cycles(lambda x: x ^ ((x>>4)&15) ^ ((x>>8)&7)))
#print('xor7', cycles(lambda x: x ^ ((x>>7)&15)))
import itertools
def cyc_fast(pos, As=range(0,2048,7)):
    tot=0
    for a in As:
        for u in range(8):
            p=pos((a*E[u])&2047)
            for g in groups:
                addrs=np.unique(p[g])
                tot+=np.bincount(addrs%16,minlength=16).max()
    return tot/(len(As)*8*4)*4
res=[]
for s1,s2 in itertools.combinations(range(4,11),2):
    f=lambda x,s1=s1,s2=s2: x ^ ((x>>s1)&15) ^ ((x>>s2)&15)
    res.append((cyc_fast(f),s1,s2))
res.sort(); print(res[:6])
