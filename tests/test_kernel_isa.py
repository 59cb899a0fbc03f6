"""ISA guard for the HIP kernels (gfx950 assembly, compiled here without a GPU).

A template or lambda change can make hipcc outline a hot loop into a real function call
(``s_swappc``) with a stack frame -- that happened once this round to ``k_hist_large``
(212 VGPRs, 848 B of scratch, boosting at a quarter of its speed) and was only caught by a
benchmark.  This test compiles every kernel file to assembly and fails on any call, and on
scratch use beyond the known, measured cases (csrc/kernels/forest.hip notes the wave-tier
row-window spill; the others are cold paths)."""
import os
import re
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "cs230_distributed_machine_learning_amd", "csrc", "kernels")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# kernel (mangled-name substring) -> scratch bytes it may use
SCRATCH_OK = {
    "k_nodesILi64ELi1E": 72,      # wave tier, binary: row-window prefetch at the 128-VGPR cap
    "k_nodesILi256ELi1E": 12,     # block tier, binary: partition row ids kept from pass 1
    "k_nodesILi128ELi1E": 12,     # the same kernel at 2 waves per node (binary builds' block tier)
    "k_dp_split_wave": 160,       # row-sharded forest: per-lane candidate arrays
    "k_dp_split": 560,
    "k_gb_gradILi64E": 528,       # multinomial boosting gradient with K > 8 classes
}


def _compile(src: str, out_dir: str) -> str:
    out = os.path.join(out_dir, os.path.basename(src) + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", KDIR, "--cuda-device-only", "-S",
                    src, "-o", out], check=True, capture_output=True, timeout=900)
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_kernel_calls_and_no_unexpected_scratch():
    srcs = sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".hip"))
    with tempfile.TemporaryDirectory() as td:
        with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
            asms = list(ex.map(lambda s: _compile(s, td), srcs))
        bad_calls, bad_scratch, kernels = [], [], 0
        for asm in asms:
            text = open(asm).read()
            if "s_swappc" in text:
                bad_calls.append(os.path.basename(asm))
            for m in re.finditer(r"\.name:\s+(\S+)\n(?:(?!\n\s+- \.).)*?\.private_segment_fixed_size:\s+(\d+)",
                                 text, re.S):
                kernels += 1
                name, scratch = m.group(1), int(m.group(2))
                if scratch == 0:
                    continue
                limit = next((v for k, v in SCRATCH_OK.items() if k in name), 0)
                if scratch > limit:
                    bad_scratch.append((name, scratch, limit))
    assert kernels > 50
    assert not bad_calls, f"kernels calling functions in {bad_calls}"
    assert not bad_scratch, f"unexpected scratch use: {bad_scratch}"
