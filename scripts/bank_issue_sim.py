#!/usr/bin/env python3
"""Simulation: can a data-dependent issue order of the 16 window adds
per lane lower the k = 8 ds_add_u32 bank-conflict cost?  Expected LDS-array cycles per
32-lane group and instruction (max bank load; bank = word mod 32 = bases j, j+1 and
the low bit of base j+2 of the window) for random bases:
  baseline (instruction j = window j)                      3.54
  half-split (lanes 0-15 issue bank bit 4 = 0 first, ...)   3.55
  pair-swap (window j or j+8 first by bank bit 4)           3.52
  full per-lane sort by bank, rotated to start at bank >= lane  3.36
The best of these (a 16-element sorting network per lane, ~120 VALU per tile, i.e.
the kernel's VALU doubled) saves 5 % of the LDS cycles: not adopted."""
import numpy as np
rng=np.random.default_rng(1)
T=4000
def cost(banks):  # banks: [T, 16 instr, 32 lanes] -> mean total cycles per 16 instructions
    c=0
    for t in range(banks.shape[0]):
        for j in range(16):
            c+=np.bincount(banks[t,j],minlength=32).max()
    return c/banks.shape[0]
# per lane: 16 windows of a random base sequence (bank = low 5 bits of 8-mer code: bases j,j+1 + low bit of j+2)
def lane_banks():
    seq=rng.integers(0,4,(T,32,32))  # T groups, 32 lanes, 32 bases
    w=np.zeros((T,32,16),np.int64)
    for j in range(16):
        w[:,:,j]=seq[:,:,j]+4*seq[:,:,j+1]+16*(seq[:,:,j+2]&1)
    return w
W=lane_banks()
base=cost(W.transpose(0,2,1)); print("baseline", base/16)
# scheme B: lanes 0-15 issue windows with bank bit4==0 first, lanes 16-31 bit4==1 first (stable order)
WB=np.empty_like(W)
for l in range(32):
    key=((W[:,l,:]>>4)&1) ^ (1 if l>=16 else 0)
    order=np.argsort(key,axis=1,kind='stable')
    WB[:,l,:]=np.take_along_axis(W[:,l,:],order,axis=1)
print("half-split", cost(WB.transpose(0,2,1))/16)
# scheme C: full sort by bank, rotated to start at bank >= l
WC=np.empty_like(W)
for l in range(32):
    s=np.sort(W[:,l,:],axis=1)
    start=(s< l).sum(axis=1)
    idx=(np.arange(16)[None,:]+start[:,None])%16
    WC[:,l,:]=np.take_along_axis(s,idx,axis=1)
print("sorted-rotated", cost(WC.transpose(0,2,1))/16)
# scheme D: pair swap: for (j, j+8) lane issues the one with bit4 == (l>=16) first
WD=W.copy()
for l in range(32):
    want=1 if l>=16 else 0
    a=WD[:,l,:8].copy(); b=WD[:,l,8:].copy()
    sw=((a>>4)&1)!=want
    WD[:,l,:8]=np.where(sw,b,a); WD[:,l,8:]=np.where(sw,a,b)
print("pair-swap", cost(WD.transpose(0,2,1))/16)
