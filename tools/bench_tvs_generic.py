import sys, os, time, json, numpy as np, torch
sys.path.insert(0, os.getcwd())
import gpsig_amd
from gpsig_amd import ops
def timed(fn, reps=5):
    fn(); torch.cuda.synchronize(); ts=[]
    for _ in range(reps):
        t0=time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter()-t0)
    return sorted(ts)[len(ts)//2]*1e3
rng=np.random.default_rng(0)
T,N,L,D,M=512,4096,100,5,5; LT=M*(M+1)//2
X=torch.tensor(np.cumsum(rng.standard_normal((N,L,D)),1)/np.sqrt(L*D),device="cuda",dtype=torch.float32)
Z=torch.tensor(rng.standard_normal((LT,T,D)),device="cuda",dtype=torch.float32)
out={}
out["tvs_linear_ms"]=timed(lambda: ops.tens_vs_seq(Z,X,M,1,"linear"))
out["tvs_rbf_order2_ms"]=timed(lambda: ops.tens_vs_seq(Z,X,M,2,"rbf"))
Xs=X[:256, :64]; Zs=Z[:, :64]*0.3
out["rescaled_ms_n256_t64_l64"]=timed(lambda: ops.rescaled(Zs, Xs, M, "linear"))
print(json.dumps(out))
