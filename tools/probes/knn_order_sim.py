"""Tile pruning of the kNN pass by spatial order (numpy count, no GPU):
the tiles of 64 consecutive particles each wave of R rows must stream at the
final (exact k-th neighbour) thresholds, Morton vs Hilbert order, at C4's
shape (N = 2e5, d = 6, k = 50, a Gaussian population with per-dimension
scales 0.5 .. 2).  Measured: R = 4: Morton 377, Hilbert 238 tiles per wave
(a kd-tree leaf order: 114; ranks per dimension + Hilbert: 191).

    python tools/probes/knn_order_sim.py R"""
import numpy as np, sys
from scipy.spatial import cKDTree
rng=np.random.default_rng(1)
N,d,k=200000,6,50
R=int(sys.argv[1])
X=rng.normal(size=(N,d))*np.linspace(0.5,2.0,d)
tau=cKDTree(X).query(X,k+1)[0][:,-1]**2
def quant(X,b):
    lo=X.min(0);hi=X.max(0)
    return np.floor((X-lo)/(hi-lo)*((1<<b)-1)).astype(np.int64)
def hilbert(X,b=10):
    x=quant(X,b).T.copy()  # d x N
    n=d; M=1<<(b-1)
    # Skilling: inverse undo excess work
    Q=M
    while Q>1:
        P=Q-1
        for i in range(n):
            m=(x[i]&Q)!=0
            # if bit set: invert low bits of x[0]
            x[0]=np.where(m, x[0]^P, x[0])
            t=(x[0]^x[i])&P
            t=np.where(m,0,t)
            x[0]^=t; x[i]^=t
        Q>>=1
    # Gray encode
    for i in range(1,n): x[i]^=x[i-1]
    t=np.zeros(x.shape[1],np.int64); Q=M
    while Q>1:
        t=np.where((x[n-1]&Q)!=0, t^(Q-1), t); Q>>=1
    for i in range(n): x[i]^=t
    key=np.zeros(x.shape[1],np.uint64)
    for bit in range(b-1,-1,-1):
        for j in range(n):
            key=(key<<np.uint64(1))|((x[j]>>bit)&1).astype(np.uint64)
    return np.argsort(key,kind='stable')
def morton(X,b=10):
    q=quant(X,b).astype(np.uint64)
    key=np.zeros(len(X),np.uint64)
    for bit in range(b-1,-1,-1):
        for j in range(d):
            key=(key<<np.uint64(1))|((q[:,j]>>np.uint64(bit))&np.uint64(1))
    return np.argsort(key,kind='stable')
for name,perm in (("morton",morton(X)),("hilbert",hilbert(X))):
    Xs=X[perm]; T=(N+63)//64
    lo=np.array([Xs[t*64:(t+1)*64].min(0) for t in range(T)]); hi=np.array([Xs[t*64:(t+1)*64].max(0) for t in range(T)])
    ts=tau[perm]; tot=0; W=0
    for w0 in range(0,N,R*50):
        rows=Xs[w0:w0+R]; tr=ts[w0:w0+R]
        need=np.zeros(T,bool)
        for r in range(len(rows)):
            dd=np.maximum(np.maximum(lo-rows[r],rows[r]-hi),0); need|=(dd**2).sum(1)<tr[r]
        tot+=need.sum(); W+=1
    print(name,R,"mean tiles/wave",tot/W,"tiles/row",tot/W/R)
