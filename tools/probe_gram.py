import sys, time, torch, numpy as np
sys.path.insert(0, '/root/repo')
import bench
from multi_fidelity_gpflow_amd.engine import Engine
eng = Engine.get(torch.device('cuda', 0))
X, Y, Xt, Yt = bench.load_goku()
Xd = torch.tensor(X, device='cuda'); n = X.shape[0]; d = X.shape[1]-1
theta = torch.tensor([1.0]+[1.0]*d+[1.0]+[1.0]*d+[1.0, 1e-3], dtype=torch.float64, device='cuda')
K = torch.empty(n, n, dtype=torch.float64, device='cuda')
for _ in range(3): eng.mf_gram(Xd, Xd, theta)
torch.cuda.synchronize()
s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(50): eng.mf_gram(Xd, Xd, theta)
e.record(); torch.cuda.synchronize()
print("dense mf_gram (Goku 1164^2):", s.elapsed_time(e)/50*1e3, "us")
