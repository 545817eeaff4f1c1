"""Round 6: units, 64-product windows and steps of k_num2 when its 64-entry
units are also cut where their entries' B rows cross one of P
product-balanced slices of B (the B-slice queues measured and dropped in
DESIGN.md §4g).  Reads rp.bin / col.bin as tools/l2sim.c does; prints, per P,
the units, windows and steps at K = 4 / 2 / 1 windows per step with the lane
utilisation (products / lanes issued)."""
import numpy as np
rp=np.fromfile('rp.bin',dtype=np.int64); col=np.fromfile('col.bin',dtype=np.int32)
n=len(rp)-1; blen=np.diff(rp)
rows=np.repeat(np.arange(n),blen)
bl=blen[col].astype(np.int64)
prodrow=np.zeros(n,np.int64); np.add.at(prodrow,rows,bl)
stream=prodrow>256
# product offset of each entry within its row
cs=np.cumsum(bl)-bl
rowstart_e=rp[:-1]
poff=np.zeros(n,np.int64); 
first=cs[rowstart_e[blen>0]]; poff[blen>0]=first
rel=cs-poff[rows]
erel=np.arange(len(col))-rp[rows]
w=np.bincount(col,weights=bl,minlength=n)
cw=np.concatenate([[0],np.cumsum(w)])
sel=stream[rows]&(bl>0)
for P in (1,8,16,32,64):
    tgt=np.arange(P+1)*cw[-1]/P
    bnd=np.searchsorted(cw,tgt); bnd[0]=0; bnd[-1]=n
    part=np.searchsorted(bnd,col,side='right')-1
    start=(erel%64==0)|np.concatenate([[True],part[1:]!=part[:-1]])|np.concatenate([[True],rows[1:]!=rows[:-1]])
    start&=sel
    # sub-unit ids: for selected entries
    idx=np.nonzero(sel)[0]
    st=start[idx]
    uid=np.cumsum(st)-1
    nu=uid[-1]+1
    pa=np.full(nu,np.iinfo(np.int64).max); pb=np.zeros(nu,np.int64)
    np.minimum.at(pa,uid,rel[idx]); np.maximum.at(pb,uid,rel[idx]+bl[idx])
    wins=((pb-1)>>6)-(pa>>6)+1
    prods=pb-pa
    res=[]
    for K in (4,2,1):
        steps=(wins+K-1)//K
        res.append('K%d steps %.2fM util %.3f'%(K,steps.sum()/1e6,prods.sum()/(64*K*steps.sum())))
    print('P=%2d units %.2fM prods/unit %.0f windows %.2fM'%(P,nu/1e6,prods.mean(),wins.sum()/1e6),' | '.join(res))
