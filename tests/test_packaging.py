"""Client packaging (reference C3: DistributedLibrary/setup.py:1-21, pyproject.toml:1-16):
``pip install .`` installs ``distributed_ml`` and the engine package (native libraries
built by the install step), and ``from distributed_ml import MLTaskManager`` works from
any directory."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_pip_install_then_import_from_elsewhere(tmp_path):
    target = tmp_path / "site"
    res = subprocess.run([sys.executable, "-m", "pip", "install", "--no-build-isolation", "--no-deps", "--target",
                          str(target), "-q", ROOT], capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stdout + res.stderr
    assert (target / "distributed_ml").is_dir() and (target / "cs230_distributed_machine_learning_amd" / "lib").is_dir()
    code = ("from distributed_ml import MLTaskManager; import cs230_distributed_machine_learning_amd as m; "
            "import os; print(MLTaskManager.__name__, os.path.dirname(m.__file__))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=str(tmp_path),
                         env=dict(os.environ, PYTHONPATH=str(target)), timeout=120)
    assert out.returncode == 0, out.stderr
    name, where = out.stdout.split()
    assert name == "MLTaskManager" and where.startswith(str(target))
    assert any(f.endswith(".so") for f in os.listdir(target / "cs230_distributed_machine_learning_amd" / "lib"))
