#!/usr/bin/env python3
"""Replay tile timelines (tools/probe_vs_render.py inputs) with the tile order's 24 classes built on
several forms of the cost estimate (neighbour blends of the probe's tile times), to rank the forms
offline.  Usage: python3 tools/tile_est_forms.py diag.bin ...  (1920-wide frames: 240 tiles a row)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tile_sched_sim import classes, simulate
from probe_vs_render import load, blend
tx = 240
def nb(t, di, dj):
    n=len(t); i=np.arange(n); x=i%tx; y=i//tx; ny=n//tx
    xx=np.clip(x+dj,0,tx-1); yy=np.clip(y+di,0,ny-1); return t[yy*tx+xx]
def box(t, r):
    acc=np.zeros_like(t); k=0
    for di in range(-r,r+1):
        for dj in range(-r,r+1): acc+=nb(t,di,dj); k+=1
    return acc/k
ests = {
 'probe': lambda t: t,
 'rowcol max (adopted)': lambda t: blend(t, tx),
 'plus mean .5/.125': lambda t: 0.5*t+0.125*(nb(t,0,-1)+nb(t,0,1)+nb(t,-1,0)+nb(t,1,0)),
 '3x3 mean': lambda t: box(t,1),
 '3x3 .5 self': lambda t: 0.5*t+0.5*box(t,1),
 '5x5 mean': lambda t: box(t,2),
 'max(3x3 mean, self/2)': lambda t: np.maximum(box(t,1), 0.5*t),
 '3x3 max': lambda t: np.max([nb(t,a,b) for a in (-1,0,1) for b in (-1,0,1)],axis=0),
}
for p in sys.argv[1:]:
    dur, probe, rec = load(p); waves=len(np.unique(rec[:,2]))
    out=[]
    for name,f in ests.items():
        e=f(probe)
        for k,ratio in ((24,2**-0.25),):
            out.append(f"{name}: {simulate(dur, np.argsort(classes(e,k,2.0,ratio),kind='stable'), waves)/1000:.1f}")
    print(p.split('/')[-1], ' | '.join(out))
