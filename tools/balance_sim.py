#!/usr/bin/env python3
"""Model of the ECS one-lane kernel's per-block work (CPU only): the cfg4
observations sorted by decreasing y, 64-observation chunks given to 512
blocks of 256 persistent lanes (rounds per observation ~ 1 + 2.33 y), each
block's finish = its busiest lane.  Compares the static stripes
(claim_pos), boustrophedon stripes, LPT over chunks and a per-stripe greedy
assignment.  (r06: the model's 12.5 % block imbalance did not show on the
GPU, profiles/r06/claim_order/.)"""
import os
import sys, heapq, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph
S,s=bd_exit(10)
y,c=simulate_ph(S,s,1_000_000,seed=DATA_KEY)
y=np.sort(y)[::-1]
r=1.0+2.33*y   # rounds per obs (model)
N=len(y); nblk=512; ch=64; L=256
nch=(N+ch-1)//ch
def block_lists(order):
    lists=[[] for _ in range(nblk)]
    for ci in range(nch):
        lists[order(ci)].append(ci)
    return lists
def block_time(chunks):
    # lanes claim obs in order from the block's chunks; obs duration r; finish = max lane time
    seq=np.concatenate([r[ci*ch:(ci+1)*ch] for ci in chunks]) if chunks else np.zeros(0)
    h=[0.0]*L
    for d in seq:
        t=heapq.heappop(h); heapq.heappush(h,t+d)
    return max(h), seq.sum()/L
def report(name, lists):
    bt=[block_time(l) for l in lists]
    fin=np.array([b[0] for b in bt]); avg=np.array([b[1] for b in bt])
    print(f"{name:10s} max finish {fin.max():7.1f}  mean finish {fin.mean():7.1f}  ideal(mean work/lane) {avg.mean():7.1f}")
report('current', block_lists(lambda ci: ci % nblk))
report('snake', block_lists(lambda ci: (ci % nblk) if (ci//nblk)%2==0 else nblk-1-(ci%nblk)))
# LPT over chunks (greedy: chunk to the least-loaded block, in decreasing order)
cw=np.array([r[ci*ch:(ci+1)*ch].sum() for ci in range(nch)])
loads=[(0.0,b) for b in range(nblk)]; heapq.heapify(loads); lists=[[] for _ in range(nblk)]
for ci in range(nch):
    l,b=heapq.heappop(loads); lists[b].append(ci); heapq.heappush(loads,(l+cw[ci],b))
report('lpt', lists)
# stripe-greedy: within each stripe, the i-th largest chunk goes to the i-th least-loaded block
load=np.zeros(nblk); lists=[[] for _ in range(nblk)]
for s0 in range(0, nch, nblk):
    cs=list(range(s0, min(nch, s0+nblk)))       # already decreasing work within the stripe
    order=np.argsort(load, kind='stable')[:len(cs)]
    for ci,b in zip(cs, order):
        lists[b].append(ci); load[b]+=cw[ci]
report('stripegrd', lists)
