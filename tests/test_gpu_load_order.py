"""One HIP runtime per process, whatever is imported first (VERDICT r05 item 3,
INTEGRATION.md "One HIP runtime per process").

torch's bundled libamdhip64.so and /opt/rocm's libamdhip64.so.7 share a
soname, so the loader binds libsgm_hip.so to whichever copy is already in the
process.  `_capi.lib()` imports torch first, so a caller that imports
stereo_matching_amd before torch still gets one runtime and a torch that sees
the GPU.  Each case runs in a fresh interpreter (the order is per process)."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PACKAGE_FIRST = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import stereo_matching_amd as sam            # the package first: nothing else loaded yet
from stereo_matching_amd import SGM, _capi, synthetic
lib = _capi.lib()                            # libsgm_hip.so now in the process
rts = _capi.hip_runtimes()
assert len(rts) == 1 and "/torch/lib/" in rts[0], rts
import torch                                 # then torch and its device tensors
assert torch.cuda.device_count() >= 1, "torch finds no GPU"
dev = torch.device("cuda", 0)
import oracle
h, w, D = 64, 200, 64
left, right = synthetic.stereo_pair(h, w, D, pair_index=3, kind="road")
L = torch.from_numpy(left).to(dev)
R = torch.from_numpy(right).to(dev)
out = torch.empty((h, w), dtype=torch.float32, device=dev)
with SGM(h, w, 1, D, device=0) as sgm:
    sgm.process_device(L.data_ptr(), R.data_ptr(), out.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize(dev)
    sgm.check()
ref = oracle.process(left, right, D)
assert np.array_equal(out.cpu().numpy().view(np.uint32), ref["lr"].view(np.uint32)), "LR map"
assert _capi.hip_runtimes() == rts, _capi.hip_runtimes()
print("package first ok", rts[0])
"""

TORCH_FIRST = r"""
import sys
sys.path.insert(0, sys.argv[1])
import torch
torch.cuda.init()
from stereo_matching_amd import _capi
_capi.lib()
rts = _capi.hip_runtimes()
assert len(rts) == 1 and "/torch/lib/" in rts[0], rts
print("torch first ok", rts[0])
"""


@pytest.mark.gpu
@pytest.mark.parametrize("script", [PACKAGE_FIRST, TORCH_FIRST], ids=["package_first", "torch_first"])
def test_one_runtime_any_import_order(script):
    r = subprocess.run([sys.executable, "-c", script, ROOT], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and " ok " in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_runtime_bound_before_library_cpu():
    # the CPU side of the same rule: after lib(), exactly one libamdhip64 is
    # mapped, and it is torch's (no device is touched)
    script = ("import sys; sys.path.insert(0, sys.argv[1]); from stereo_matching_amd import _capi; "
              "_capi.lib(); r = _capi.hip_runtimes(); "
              "assert len(r) == 1 and '/torch/lib/' in r[0], r; print('cpu ok', r[0])")
    r = subprocess.run([sys.executable, "-c", script, ROOT], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "cpu ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
