"""Bound LKRefine's fp32 evaluation order.

Runs tools/lk_orders.c's restatement of LKRefine under five evaluation orders
of its Eigen reductions on the K128 and 4K fixtures (synthetic pairs through
the oracle's SGM + LR + post_filter: the map LKRefine refines in config 5)
and reports, against the index order the oracle and the GPU use: max |delta
disp|, pixels above north_star's 1e-4, and pixels whose iteration count or
exit test differs (a break test that flipped).  Writes the table to
profiles/r03_lk_orders.txt.  CPU only; test infrastructure like oracle/.
Usage: python tools/lk_orders.py [--no-4k]
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from stereo_matching_amd import synthetic  # noqa: E402

ORDERS = ["index (oracle, GPU)", "Eigen SSE2 Packet4f redux", "Eigen AVX Packet8f redux",
          "pairwise", "dense-diagonal GEMV (explicit zeros) + SSE2 redux"]
EXITS = ["none", "10 iterations", "valid < 4.9", "Hessian < 1e-3", "NaN doff", "diverged",
         "disp out of range", "converged < 1e-6"]


def build():
    out = os.path.join(ROOT, "build", "liblk_orders.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c11", "-fPIC", "-fopenmp", "-ffp-contract=off",
                    "-fno-fast-math", "-shared", "-o", out, os.path.join(ROOT, "tools", "lk_orders.c"),
                    "-lm"], check=True)
    lib = ctypes.CDLL(out)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.lk_refine_order.argtypes = [P, P, P, I, I, I, I, P, P]
    return lib


def run(lib, L, R, disp, D, order):
    H, W = disp.shape
    F = np.array(disp, np.float32, copy=True, order="C")
    it = np.empty((H, W), np.int32)
    ex = np.empty((H, W), np.int32)
    lib.lk_refine_order(L.ctypes.data, R.ctypes.data, F.ctypes.data, H, W, D, order,
                        it.ctypes.data, ex.ctypes.data)
    return F, it, ex


def fixture(name):
    if name == "K128":
        h, w, D = 375, 1242, 128
        left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
        ref = oracle.process(left, right, D)
    else:
        from test_gpu_fullsize import _config5_images
        h, w, D = 2160, 3840, 256
        left, right = _config5_images(h, w, 4)
        ml, mr = oracle.sky_detect(left), oracle.sky_detect(right)
        ref = oracle.process(left, right, D, sky_l=ml, sky_r=mr, schedule="lean")
    return left, right, ref["final"], D


def main():
    lib = build()
    names = ["K128"] + ([] if "--no-4k" in sys.argv else ["4K256"])
    lines = ["LKRefine under other fp32 evaluation orders of its Eigen sums",
             "(tools/lk_orders.c; LKSubPixelImpl.cpp:172-186; inputs: the oracle's post-filtered",
             " map of each fixture, as config 5 refines it)", ""]
    for name in names:
        t0 = time.time()
        left, right, final, D = fixture(name)
        base, bit, bex = run(lib, left, right, final, D, 0)
        want = oracle.lk_refine(left, right, final, D)
        assert np.array_equal(base.view(np.uint32), want.view(np.uint32)), "index order != oracle"
        refined = int(np.count_nonzero(bit > 0))
        lines.append(f"{name}: {final.shape[1]}x{final.shape[0]} D={D}, {refined} pixels iterated "
                     f"(index order reproduces orc_lk_refine bit for bit)")
        lines.append(f"  {'order':52s} {'max|dd|':>10s} {'>1e-4':>7s} {'!=bits':>8s} "
                     f"{'iters!=':>8s} {'exit!=':>7s}")
        for order in range(1, len(ORDERS)):
            got, it, ex = run(lib, left, right, final, D, order)
            fin = np.isfinite(got) & np.isfinite(base)
            dd = np.abs(got[fin].astype(np.float64) - base[fin].astype(np.float64))
            mx = float(dd.max()) if dd.size else 0.0
            over = np.argwhere(np.abs(got.astype(np.float64) - base.astype(np.float64)) > 1e-4)
            lines.append(f"  {ORDERS[order]:52s} {mx:10.3g} {len(over):7d} "
                         f"{int(np.count_nonzero(got.view(np.uint32) != base.view(np.uint32))):8d} "
                         f"{int(np.count_nonzero(it != bit)):8d} {int(np.count_nonzero(ex != bex)):7d}")
            for (i, j) in over[:6]:
                lines.append(f"      ({i},{j}): index {base[i, j]:.7g} ({bit[i, j]} it, "
                             f"{EXITS[bex[i, j]]}) vs {got[i, j]:.7g} ({it[i, j]} it, "
                             f"{EXITS[ex[i, j]]})")
        lines.append(f"  ({time.time() - t0:.0f} s)")
        lines.append("")
        print("\n".join(lines[-(len(ORDERS) + 4):]), flush=True)
    out = os.path.join(ROOT, "profiles", "r03_lk_orders.txt")
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
