#!/usr/bin/env python3
"""Flush rounds per decode tile, today (every pass flushes all its complete chunks) against a
deferred flush (whole 64-chunk rounds only, the rest staged for the next tile), over the oracle's
encodings of 8 synthetic 64 KiB buffers per kind.  CPU only; sizes DESIGN.md §4 "run-heavy kinds".
usage: python tools/flush_rounds_sim.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import rle_oracle as O  # noqa: E402   (test infrastructure: the checker's encoder)
def tile_outputs(y):
    # decoded bytes of the tokens starting in each 1008-byte tile
    C=len(y); j=0; outs={}
    while j<C:
        t=j//1008
        if j+1<C and y[j]==y[j+1]:
            n=y[j+2]-48 if j+2<C else 1; outs[t]=outs.get(t,0)+n; j+=3
        else: outs[t]=outs.get(t,0)+1; j+=1
    return [outs.get(t,0) for t in range((C+1007)//1008)]
def rounds_now(outs, cap):   # cap: pass capacity in positions (kPassCap)
    rel=0; r=0
    for o in outs:
        left=o
        while True:
            p=min(left, cap-rel) if rel+left>cap else left
            nfl=(rel+p)//16; r+=-(-nfl//64); rel=(rel+p)%16; left-=p
            if left==0: break
    return r
def rounds_defer(outs, cap):
    rel=0; r=0
    for o in outs:
        if rel+o>cap:   # pre-flush everything staged
            nfl=rel//16; r+=-(-nfl//64); rel%=16
        left=o
        while True:
            p=min(left, cap-rel) if rel+left>cap else left
            left-=p; nfl=(rel+p)//16
            if left==0:
                full=(nfl//64)*64; r+=nfl//64; rel=rel+p-16*full
                break
            r+=-(-nfl//64); rel=(rel+p)%16
    return r
for kind,name in [(2,'runs50'),(3,'runs90'),(0,'zero'),(1,'random')]:
    tot={}
    for i in range(8):
        x=O.gen(kind,i,65536); y=O.encode(x); outs=tile_outputs(y)
        for cap,cn in [(16*192-17,'192'),(16*96-17,'96')]:
            a=rounds_now(outs,cap); b=rounds_defer(outs,cap)
            tot.setdefault(cn,[0,0,0]); tot[cn][0]+=a; tot[cn][1]+=b; tot[cn][2]+=len(outs)
    print(name, {k:'now %.2f defer %.2f rounds/tile'%(v[0]/v[2],v[1]/v[2]) for k,v in tot.items()}, 'avg out/tile %.0f'%(sum(outs)/len(outs)))
