"""Per-phase cycle breakdown of k_nodes (needs a -DDML_PHASE_PROF build via DML_HIP_LIB)."""
import ctypes, sys, runpy
import numpy as np
sys.argv = ["sweep_tiers.py"]
runpy.run_path("/root/repo/scripts/sweep_tiers.py", run_name="__main__")
from cs230_distributed_machine_learning_amd.utils import native
lib = native.hip_lib()
out = np.zeros(32, dtype=np.uint64)
lib.dml_forest_phase_stats.argtypes = [ctypes.c_void_p]
rc = lib.dml_forest_phase_stats(out.ctypes.data)
names = ["setup", "feat_extract", "hist", "eval", "select", "decision", "partition", "nodes"]
for t, tn in enumerate(["wave(64)", "block"]):
    v = out[t * 8:(t + 1) * 8].astype(float)
    n = v[7] or 1
    tot = v[:7].sum()
    rows = float(out[24 + t])
    print(tn, f"nodes={int(v[7])} rows/node={rows/n:.0f} cycles/node={tot/n:.0f}", "  ".join(f"{names[i]}={v[i]/n:.0f} ({100*v[i]/tot:.0f}%)" for i in range(7)))
v = out[16:24].astype(float)
n = v[7] or 1
tot = v[:5].sum()
sn = ["setup", "seg_eval", "onefeat_eval", "split_push", "tail"]
print("subtree(64)", f"roots={int(v[7])} rows/root={float(out[26])/n:.1f} cycles/root={tot/n:.0f}",
      "  ".join(f"{sn[i]}={v[i]/n:.0f} ({100*v[i]/tot:.0f}%)" for i in range(5)),
      f"seg_nodes={int(out[28])} (rows/node {float(out[29])/max(1,out[28]):.1f}) onefeat_nodes={int(out[30])} "
      f"(rows/node {float(out[31])/max(1,out[30]):.1f})")
