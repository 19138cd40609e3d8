"""Held-Karp 1-tree bound at the root of the hardest 32-city K2 seeds (CPU
prototype of search_abi.cpp:held_karp_pi): subgradient ascent towards the
multi-start heuristic's cost or a nearest-neighbour tour's, bound / heuristic
printed.  python tools/k2_tree_bound_proto.py [seed ...]"""
import sys, numpy as np
sys.path.insert(0,'/root/repo/tsp-mpi-reduction_amd'); sys.path.insert(0,'/root/repo')
import tspgpu
from bench import k2_instance
def mst(dp, verts):
    verts=list(verts); m=len(verts)
    intree=[False]*m; key=[np.inf]*m; key[0]=0; tot=0; deg=np.zeros(len(dp),int); par=[-1]*m
    for _ in range(m):
        u=min((i for i in range(m) if not intree[i]), key=lambda i:key[i]); intree[u]=True; tot+=key[u]
        if par[u]>=0: deg[verts[u]]+=1; deg[verts[par[u]]]+=1
        for v in range(m):
            if not intree[v] and dp[verts[u],verts[v]]<key[v]: key[v]=dp[verts[u],verts[v]]; par[v]=u
    return tot, deg
def onetree(d, pi):
    n=len(d); dp=d+pi[:,None]+pi[None,:]
    t,deg=mst(dp, range(1,n))
    r=np.argsort(dp[0,1:])[:2]+1
    t+=dp[0,r[0]]+dp[0,r[1]]; deg[0]+=2; deg[r[0]]+=1; deg[r[1]]+=1
    return t-2*pi.sum(), deg
def hk(d, ub, iters=300):
    n=len(d); pi=np.zeros(n); best=(-1e300,pi); lam=2.0; stall=0
    for it in range(iters):
        lb,deg=onetree(d,pi)
        if lb>best[0]: best=(lb,pi.copy()); stall=0
        else:
            stall+=1
            if stall>=10: lam*=0.7; stall=0
        g=deg-2.0; nn=(g*g).sum()
        if nn==0: break
        pi=pi+lam*(ub-lb)/nn*g
    return best
for seed in [int(x) for x in sys.argv[1:]]:
    d=k2_instance(32,seed); h,_=tspgpu.heuristic_tour(d)
    lb,pi=hk(d,h)
    # path bound at the root: MST over all cities (path 0 -> ... -> 0 is a cycle; as path from k=0 to 0: set = all)
    print(seed, "HK 1-tree/heur", round(lb/h,4), flush=True)
def nn_ub(d):
    n=len(d); used=[0]*n; used[0]=1; k=0; s=0
    for _ in range(n-1):
        b=min((j for j in range(n) if not used[j]), key=lambda j:d[k,j]); s+=d[k,b]; used[b]=1; k=b
    return s+d[k,0]
for seed in [14,35,30]:
    d=k2_instance(32,seed); h,_=tspgpu.heuristic_tour(d)
    for it in (100,300):
        lb,pi=hk(d,nn_ub(d),it); print(seed,"nn-target",it,round(lb/h,5), flush=True)
    lb,pi=hk(d,h,300); print(seed,"h-target 300",round(lb/h,5))
