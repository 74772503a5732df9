#!/usr/bin/env python3
"""Launch-tail study: each adaptive phase's samples (scripts/adaptive_sim.py, capture) list-scheduled on
P lanes (argv[1], default 262144), one time unit per segment; the tail beyond total / P for the pixel
order, pixels ordered by their earlier samples' mean path length, and per-sample LPT.
(profiles/r05/adaptive_drain_order_sim.txt)"""
import heapq
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np, adaptive_sim as A
L,segs=A.samples('c3_bunny','/tmp/adaptive_sim_c3.npz',8)
pre=A.prepare(L,segs); del L
cap=[]
ph,nfin=A.simulate(pre,200,phase_slots=1<<21,margins=[0.8,1.25,1.5],pool=1,pool_w=8.0,width=1000,capture=cap)
P=int(sys.argv[1]) if len(sys.argv)>1 else 262144
def makespan(d):
    # list scheduling, lanes take samples in order
    n=len(d)
    if n<=P: return d.max()
    h=list(d[:P].astype(np.int64)); heapq.heapify(h)
    for x in d[P:]:
        t=heapq.heappop(h); heapq.heappush(h,t+int(x))
    return max(h)
for g,(act,n0,kk) in enumerate(cap):
    if g==0: continue
    # slot order: pixels in list (pixel) order, each pixel's samples consecutive
    rep=np.repeat(np.arange(act.size),kk)
    sidx=np.concatenate([np.arange(a,a+b) for a,b in zip(n0,kk)])
    d=segs[act[rep],sidx].astype(np.int64)
    tot=d.sum(); ideal=tot/P
    t0=time.time(); m_pix=makespan(d)
    # known cost: mean segs of the pixel's earlier samples
    mean_prev=np.array([segs[p,:a].mean() for p,a in zip(act,n0)])
    order=np.argsort(-mean_prev,kind='stable')
    d2=np.concatenate([segs[act[i],n0[i]:n0[i]+kk[i]] for i in order]).astype(np.int64)
    m_sorted=makespan(d2)
    d3=np.sort(d)[::-1]; m_lpt=makespan(d3)
    print(f"phase {g+1}: {act.size} px {d.size} samples {tot} segs ideal {ideal:.1f} | pixel order {m_pix} (+{m_pix-ideal:.1f}) | by prior mean desc {m_sorted} (+{m_sorted-ideal:.1f}) | LPT samples {m_lpt} (+{m_lpt-ideal:.1f}) | max path {d.max()} ({time.time()-t0:.0f}s)",flush=True)
