import sys, numpy as np
sys.path.insert(0,'/root/repo/tsp-mpi-reduction_amd'); sys.path.insert(0,'/root/repo')
import tspgpu
from bench import k2_instance
def two_nb(d, pi):
    n=len(d); dp = d + pi[:,None] + pi[None,:]
    np.fill_diagonal(dp, np.inf)
    idx = np.argsort(dp, axis=1)[:, :2]
    m = np.take_along_axis(dp, idx, axis=1)
    lb = m.sum()/2 - 2*pi.sum()
    cnt = np.bincount(idx.ravel(), minlength=n)
    return lb, cnt
def ascent(d, ub, iters=int(sys.argv[1]) if len(sys.argv)>1 else 2000, win=int(sys.argv[2]) if len(sys.argv)>2 else 20):
    n=len(d); pi=np.zeros(n); best=(-1e300, pi.copy()); lam=2.0; stall=0
    for it in range(iters):
        lb, cnt = two_nb(d, pi)
        if lb > best[0] + 1e-12: best=(lb, pi.copy()); stall=0
        else:
            stall+=1
            if stall>=win: lam*=0.7; stall=0
        g = cnt/2.0 - 1.0
        nn = (g*g).sum()
        if nn == 0: break
        pi = pi + lam*(ub-lb)/nn * g
    return best
for (n,seed) in [(30,2),(30,1),(28,2),(24,1)]:
    d=k2_instance(n,seed); ub,_=tspgpu.heuristic_tour(d)
    lb0,_=two_nb(d,np.zeros(n))
    lb1,pi=ascent(d,ub)
    print(n,seed,"ub",round(ub,2),"2nb",round(lb0/ub,4),"2nb+pi",round(lb1/ub,4))
for f in ['ulysses22.tsp','gr17.tsp','ulysses16.tsp']:
    _,di=tspgpu.read_tsplib('/root/repo/tests/golden/tsplib/'+f); d=di.astype(float)
    ub,_=tspgpu.heuristic_tour(di)
    lb0,_=two_nb(d,np.zeros(len(d))); lb1,pi=ascent(d,ub)
    print(f,"ub",ub,"2nb",round(lb0/ub,4),"2nb+pi",round(lb1/ub,4))
