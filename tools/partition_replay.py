#!/usr/bin/env python3
"""Replays the fused pass controller (kernels.hip adapted_bound) on the raw
arrays tools/partition_probe.py saves (OUT=gpurun_out/probe): the predicted
next bounds against the GPU's, and the targets by wave slot."""
import numpy as np, sys
NR=4096
P=[np.load(f'gpurun_out/probe/probe_{k}.npy') for k in range(6)]
B=[p[:NR+1] for p in P]; ts=[p[NR+1:2*NR+1] for p in P]; te=[p[2*NR+1:3*NR+1] for p in P]; nch=[p[3*NR+1:] for p in P]
cost=[np.clip(((te[k]-ts[k])>>2)+nch[k]*600,1,0xFFFF) for k in range(6)]
def adapt(c, rb, frm, g=1):
    cc=np.concatenate([[0],np.cumsum(c)]).astype(np.int64); tot=int(cc[-1])
    out=frm.copy()
    for k in range(1,NR):
        T=k*tot//NR
        lo=np.searchsorted(cc[:NR+1],T,side='right')-1; lo=min(lo,NR-1)
        cr=cc[lo+1]-cc[lo]
        tfp=int(rb[lo])*256+((T-cc[lo])*(int(rb[lo+1])-int(rb[lo]))*256//cr if cr else 0)
        out[k]=(int(frm[k])*256*(4-g)+tfp*g+512)>>10
    return out
for k in range(1,5):
    pred=adapt(cost[k-1],B[k-1],B[k])
    act=B[k+1]
    print(k,'max |pred-act|',np.abs(pred-act).max(),'mean|.|',np.abs(pred-act).mean().round(3),' mean|act-cur|',np.abs(act-B[k]).mean().round(3), 'mean|pred-cur|', np.abs(pred-B[k]).mean().round(3))
# what the targets look like: full-gain target vs current
k=3
tgt=adapt(cost[k-1],B[k-1],B[k],g=4)
d=(tgt-B[k])[:NR]
print('target - current by slot (iterations):', [round(d[np.arange(NR)%16==i].mean(),2) for i in range(16)])
c=cost[k].astype(float)*0.04
print('cost dev by slot (us):', [round(c[np.arange(NR)%16==i].mean()-c.mean(),2) for i in range(16)])
ln=np.diff(B[k]).astype(float)
print('len by slot', [round(ln[np.arange(NR)%16==i].mean(),2) for i in range(16)])
