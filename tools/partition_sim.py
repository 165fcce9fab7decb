#!/usr/bin/env python3
"""Simulation of the fused pass's adaptive partition:
4096 ranges, per-slot speed biases and per-workgroup speeds as measured
(profiles/r04q_partition_probe.txt), a fixed tail cost and a per-range
per-pass noise SD.  'global' is the kernel's controller (kernels.hip
adapted_bound: boundary k moves gain/4 of the way to where the previous
pass's cumulative cost curve crosses k/NR); 'local' scales each range's
length by mean cost / its cost, renormalised, with fixed-point state.
Prints the residual slot biases (slots 0, 11, 12), the mean of the max range
cost above the mean, and the workgroup maxima.
usage: python tools/partition_sim.py"""
import numpy as np
NR=4096; IT=150000128//512
def run(mode, g=1, passes=200, seed=0, SD=1.5, fixed=7.0):
    rng=np.random.default_rng(seed)
    slot=np.tile(np.array([-2.2,-.7,-.3,-.3,.2,.2,.2,.6,-1,-.7,-1,-2.3,2.5,1.5,1.3,2])/68+1,NR//16)
    wgs=1+rng.normal(0,0.02,256).repeat(16)   # persistent per-WG speed
    def costs(b):
        ln=np.diff(b).astype(float)
        return ln*(66.0/(IT/NR))*slot*wgs + fixed + rng.normal(0,SD,NR)
    pos=np.linspace(0,IT,NR+1)*256
    b=np.round(pos/256).astype(np.int64)
    prev=b.copy(); cprev=costs(b)
    hist=[]
    for p in range(passes):
        c=costs(b)
        if mode=='global':
            cc=np.concatenate([[0],np.cumsum(cprev)]); tot=cc[-1]
            T=np.arange(NR+1)*tot/NR
            lo=np.clip(np.searchsorted(cc,T,side='right')-1,0,NR-1)
            cr=cc[lo+1]-cc[lo]
            tfp=(prev[lo]+(T-cc[lo])*(prev[lo+1]-prev[lo])/cr)*256
            npos=(b*256.0*(4-g)+tfp*g)/4
        else:
            lp=np.diff(prev).astype(float)          # lengths the costs were measured over
            tgt=lp*cprev.mean()/np.maximum(cprev,1e-9)
            lc=np.diff(pos)/256.0                   # current lengths (fixed point)
            nl=lc*(4-g)/4+tgt*g/4
            npos=np.concatenate([[0],np.cumsum(nl)])*IT/np.sum(nl)*256
        npos[0]=0; npos[-1]=IT*256
        nb=np.round(npos/256).astype(np.int64)
        cprev=c; prev=b; b=nb; pos=npos
        if p>=passes-30: hist.append(costs(b))
    h=np.array(hist); d=h-h.mean(1,keepdims=True)
    sl=[round(d[:,i::16].mean(),2) for i in range(16)]
    wgmax=h.reshape(len(h),256,16).max(2)
    return [sl[0],sl[11],sl[12]], 'max-mean', round(float(np.mean(h.max(1)-h.mean(1))),2), 'WGmax max-med', round(float(np.mean(wgmax.max(1)-np.median(wgmax,1))),2), 'WGmax p50-mean', round(float(np.mean(np.median(wgmax,1)-h.mean(1))),2)
for SD in (1.5, 3.5):
    for mode in ('global', 'local'):
        for g in (1, 2):
            print(mode, 'g', g, 'SD', SD, run(mode, g, SD=SD))
