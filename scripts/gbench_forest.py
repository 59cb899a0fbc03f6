import numpy as np, torch, time, sys, os
sys.path.insert(0, '/root/repo')
from cs230_distributed_machine_learning_amd.ops import binning, forest_ops
from cs230_distributed_machine_learning_amd.utils import native
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles
dev = torch.device('cuda:0')
n, d = int(sys.argv[1]), int(sys.argv[2]); ntrees=int(sys.argv[3]); nfits=int(sys.argv[4]); depth=int(sys.argv[5]) if len(sys.argv)>5 else 2**31-1
g = torch.Generator(device=dev); g.manual_seed(0)
X = torch.randn(n, d, device=dev, generator=g)
w = torch.randn(d, device=dev, generator=g) * (torch.arange(d, device=dev) < 20)
y = ((X @ w + 0.5*torch.randn(n, device=dev, generator=g)) > 0).to(torch.int32)
t0=time.time(); edges = binning.quantile_edges(X); Xb = binning.bin_matrix(X, edges); torch.cuda.synchronize(); print('bin', time.time()-t0)
roles, _ = make_split_roles(y.cpu().numpy(), 5, True, holdout=False)
roles = torch.from_numpy(roles).to(dev)
specs = forest_ops.make_specs(nfits*ntrees)
for f in range(nfits):
    for t in range(ntrees):
        s = specs[f*ntrees+t]; s['seed']=7+t+1000*f; s['split']=f%5; s['fit']=f; s['max_depth']=depth; s['min_samples_split']=2; s['min_samples_leaf']=1
        s['max_features']=int(np.sqrt(d)); s['bootstrap']=1; s['criterion']=0; s['pois_cdf']=native.poisson_cdf_table(1.0)
for rep in range(2):
    torch.cuda.synchronize(); t0=time.time()
    XbT = None if os.environ.get('DML_NO_XBT') else Xb[:, :d].t().contiguous()   # the family path's feature-major copy
    fb = forest_ops.build_gpu(Xb, y, None, roles, specs, 2, False, XbT=XbT)
    torch.cuda.synchronize(); t1=time.time()
    print('build', t1-t0, fb.stats, 'per-tree ms', (t1-t0)/len(specs)*1e3)
rows=[]; roff=[0]
for f in range(nfits):
    r = torch.nonzero(roles[f%5]==2).flatten().to(torch.int32); rows.append(r); roff.append(roff[-1]+len(r))
rows = torch.cat(rows); roff=np.array(roff); toff=np.arange(nfits+1)*ntrees
torch.cuda.synchronize(); t0=time.time()
pred = forest_ops.predict(fb, Xb, toff, roff, rows)
st = forest_ops.score_stats(rows, roff, pred, ycls=y)
torch.cuda.synchronize(); print('predict+score', time.time()-t0, 'acc', st[:,0]/st[:,3])
