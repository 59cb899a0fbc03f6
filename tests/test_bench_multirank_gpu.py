"""bench.py's N>1 path on the one-GPU test box: two ranks share device 0 over gloo
(DML_SHARE_DEVICE / DML_DIST_BACKEND rehearsal knobs; on an 8-GPU node the same code
runs one rank per GPU over RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_bench_two_ranks_share_one_gpu():
    env = dict(os.environ, DML_SHARE_DEVICE="1", DML_DIST_BACKEND="gloo", DML_HBM_BUDGET_GB="20",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rows", "62500", "--features", "20",
           "--cands-per-rank", "2", "--cv", "3", "--steps", "1", "--warmup", "1", "--master-port", str(_free_port())]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["steps"] == 1 and rec["config"]["global_batch"] == 2 * 2 * 3
    assert rec["value"] > 0 and 0.5 < rec["mean_cv_accuracy_last_step"] <= 1.0
