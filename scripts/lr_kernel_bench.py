#!/usr/bin/env python3
"""Per-kernel timing of the MFMA logistic objective (forward / gradient launches separately).
A/B variants of libdml_hip.so are selected with DML_HIP_LIB."""
import ctypes, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from cs230_distributed_machine_learning_amd.data import synthetic
from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.models import linear
from cs230_distributed_machine_learning_amd.models.base import FitTask
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles
from cs230_distributed_machine_learning_amd.utils import native

rows, d, fits = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2_000_000, 1000, 512)))
dev = torch.device("cuda:0")
X, y = synthetic.make_table(rows, d, informative=10, n_classes=2, noise=1.0, seed=1, device=dev, block=rows // 8)
dd = DeviceData(X, y, True, dev)
roles, names = make_split_roles(y.cpu().numpy(), 5, True, holdout=False, test_size=0.2, random_state=0)
dd.set_splits(roles, names)
fam = linear.LogisticFamily()
tasks = [FitTask(task_id=i, candidate=i, split=i % 5, model_type="LogisticRegression",
                 params=fam.resolve("LogisticRegression", {"C": 1.0}, dd.n, dd.d, 2)) for i in range(fits)]
b = linear._Batch(dd, tasks)
W = torch.randn((d + 1, b.M), device=dev) * 0.01
b.mf = linear.MfmaPlan(dd, b)
b.mf.objective(dd, b, W)
lib = native.hip_lib()
st = native.stream_handle(dev)
out = {"lib": os.path.basename(os.environ.get("DML_HIP_LIB", "default")), "v3": bool(b.mf.v3), "Mp": b.mf.Mp}
if b.mf.v3:   # row chunks: (forward, gradient) launches per chunk
    calls = {"fwd": [(lib.dml_lr_mfma_fwd3, a) for a in b.mf.fwd_l],
             "grad": [(lib.dml_lr_mfma_grad3, a) for a in b.mf.grad_l]}
    out["chunks"] = b.mf.n_chunks
else:
    calls = {"fwd": [(lib.dml_lr_mfma_fwd, b.mf.fwd)], "grad": [(lib.dml_lr_mfma_grad, b.mf.grad)]}
for name, lst in calls.items():
    for fn, args in lst:
        rc = fn(ctypes.byref(args), st)
        assert rc == 0, (name, rc)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        for fn, args in lst:
            fn(ctypes.byref(args), st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    out[name + "_ms"] = round(ms, 3)
    out[name + "_tflops_bf16"] = round(3 * 2 * rows * 1024 * b.mf.Mp / ms / 1e9, 1)
print(json.dumps(out), flush=True)
