#!/usr/bin/env python3
"""How often two samples of one pixel quadrant walk the same cells (planning
estimate for two samples per lane, DESIGN.md 8 Next; CPU only).

    python tools/pair_coherence.py [config=c5] [pixels=300]

Random pixels; per pixel two pairs of jittered samples from the same jitter
quadrant; each ray's depth-K grid cells (a float64 3D DDA over the table's
grid, K = 6 for C5, 5 for C5d) from the root box to its oracle hit; reports
|shared| / |union| of the two cell sets.  A proxy: the walk visits leaves,
which sit at or above depth K on these trees.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, oracle, raytracingstudy_amd as rt
from raytracingstudy_amd.camera import scene_pose
rng=np.random.default_rng(1)
CFG=sys.argv[1] if len(sys.argv)>1 else 'c5'; NPIX=int(sys.argv[2]) if len(sys.argv)>2 else 300
c=rt.CONFIGS[CFG]; W,H=c.width,c.height
sp,al=rt.configs.scene_spheres(c, rt.SEED)
sc=oracle.Scene(sp,al,max_depth=c.max_depth,leaf_capacity=c.leaf_capacity)
pose=scene_pose(); K=oracle.resize_intrinsic(W,H)
P=np.asarray(pose,np.float64).reshape(4,4); o=P[3,:3] if abs(P[3,3]-1)<1e-9 and np.any(P[3,:3]) else P[:3,3]
Kc={'c5':6,'c5d':5,'c3':5}.get(CFG,6); G=1<<Kc; lo=np.zeros(3); ext=1.28
def cells(o,d,tmax):
    # grid DDA over the depth-K grid from the box entry to tmax
    inv=1/np.where(np.abs(d)<1e-20,1e-20,d)
    t0=np.max(np.minimum((lo-o)*inv,(lo+ext-o)*inv)); t1=np.min(np.maximum((lo-o)*inv,(lo+ext-o)*inv))
    t0=max(t0,0); t1=min(t1,tmax)
    if t0>=t1: return []
    p=o+d*(t0+1e-9); cell=np.clip(((p-lo)/ext*G).astype(int),0,G-1); out=[]
    step=np.sign(d).astype(int); t=t0
    nxt=lambda i: ((cell[i]+(step[i]>0))*ext/G+lo[i]-o[i])*inv[i]
    while t<t1 and len(out)<4*G:
        out.append(tuple(cell))
        tn=[nxt(i) if step[i]!=0 else np.inf for i in range(3)]
        i=int(np.argmin(tn)); t=tn[i]; cell[i]+=step[i]
        if cell[i]<0 or cell[i]>=G: break
    return out
share=[];
for _ in range(NPIX):
    x,y=rng.integers(0,W),rng.integers(0,H)
    for s in range(2):
        u1,v1=x+rng.random(),y+rng.random()
        # a second sample of the same pixel quadrant
        qx,qy=int((u1-x)*2),int((v1-y)*2)
        u2,v2=x+(qx+rng.random())/2,y+(qy+rng.random())/2
        seqs=[]
        for (u,v) in ((u1,v1),(u2,v2)):
            d=oracle.get_ray(pose,K,u,v).astype(np.float64)
            hit,t,idx,_=sc.trace(o.astype(np.float32),d.astype(np.float32))
            seqs.append(cells(o,d,t if hit else np.inf))
        a,b=set(seqs[0]),set(seqs[1])
        if a|b: share.append(len(a&b)/len(a|b))
share=np.array(share)
print(CFG,'K',Kc,'pairs',len(share),'mean shared/union cells',share.mean().round(3),'p10',np.percentile(share,10).round(3),'median',np.median(share).round(3))
