"""Hop timeline of the slanted passes: when
each tile's exit states were stored, when the next tile's receiver needed and
held them, and when compute wave 0 published each step (s_memrealtime,
100 MHz, chip-wide).  Round 6's passes have no per-step barrier (DESIGN.md 5e
"Dataflow"): "lead" is how long before the consumer's phase began the
producer had issued the states it needs -- positive when the exits were
produced ahead of their consumer.

Library built with -DSGM_SLANT_HOPS (bash tools/variant.sh hops
-DSGM_SLANT_HOPS), loaded with SGM_HIP_LIB=build/hops/libsgm_hip.so.
Usage (GPU): python tools/slant_hops.py [H W D V]   (default HD256, two views)

Printed per pass:
  * hop: held(t, s) - stored(t+1, s), the producer's store to the consumer
    holding the states, over the phases in which the receiver had to wait
    (held - needed > 0.2 us) and over all phases;
  * wait: held - needed, the time the receiver's phase waited for the hop;
  * lead: needed(t, s) - stored(t+1, s), the producer's head start;
  * step: published(t, s) - published(t, s-1), wave 0's step period, split
    by whether the step's input hop made the receiver wait;
  * lag: published(t, s) - published(t+1, s-1), how far a tile runs behind
    its producer."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SGM_SLANT"] = "1"
import torch  # noqa: E402

from stereo_matching_amd import SGM, _capi, synthetic  # noqa: E402

NW, NW_UP = 14, 15  # tile widths: top-down, bottom-up (sgm_internal.h)


def pct(x):
    if x.size == 0:
        return "n/a"
    q = np.percentile(x, [10, 50, 90])
    return f"p10 {q[0]:6.2f}  p50 {q[1]:6.2f}  p90 {q[2]:6.2f}  mean {x.mean():6.2f} us  (n={x.size})"


def main():
    h, w, D, V = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (1080, 1920, 256, 2)
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    dev = torch.device("cuda", 0)
    dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
    out = torch.empty((h, w), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    sgm = SGM(h, w, 1, D, views=V, device=0)
    lib = _capi.lib()
    lib.sgm_debug_slant_hops.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    TS = {0: (w + h - 1 + NW - 1) // NW, 1: (w + h - 1 + NW_UP - 1) // NW_UP}  # per pass
    n = V * max(TS.values()) * h
    for _ in range(3):
        sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
    sgm.check()
    assert lib.sgm_debug_slant_hops(None, n, 1) == 0
    sgm.set_profiling(True)
    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
    sgm.check()
    prof = sgm.get_profile()
    buf = np.zeros((2, 4, n), np.uint32)
    assert lib.sgm_debug_slant_hops(buf.ctypes.data, n, 0) == 0
    print(f"{w}x{h} D={D} V={V}: {TS[0]} / {TS[1]} tiles per view (top-down / bottom-up); slant_down {prof['slant_down'][1]:.3f} ms, "
          f"slant_up {prof['slant_up'][1]:.3f} ms")
    for p, name in ((0, "top-down"), (1, "bottom-up")):
        T = TS[p]
        a = buf[p][:, :V * T * h].reshape(4, V, T, h).astype(np.int64)
        have = a != 0
        t0 = a[have].min()

        def us(x):
            return (x % (1 << 32)).astype(np.float64) / 100.0  # ticks (10 ns) -> us

        st, nd, hd, br = a[0], a[1], a[2], a[3]
        # consumer tile t, step s needs producer tile t+1's step s (its exit states)
        ok = have[1][:, :-1, :] & have[2][:, :-1, :] & have[0][:, 1:, :]
        hop = us((hd[:, :-1, :] - st[:, 1:, :]) % (1 << 32))[ok]
        wait = us((hd[:, :-1, :] - nd[:, :-1, :]) % (1 << 32))[ok]
        waited = wait > 0.2
        print(f"  {name}: span {us(np.array([a[have].max() - t0]))[0]:.0f} us, phases {ok.sum()}, "
              f"receiver waited in {waited.mean() * 100:.1f}%")
        print(f"    hop  (waited) {pct(hop[waited])}")
        print(f"    hop  (all)    {pct(hop)}")
        print(f"    wait (waited) {pct(wait[waited])}")
        lead = us((nd[:, :-1, :] - st[:, 1:, :]) % (1 << 32))
        lead = np.where(lead > 2 ** 31 / 100, lead - 2 ** 32 / 100, lead)[ok]
        print(f"    lead (consumer needs - producer stored) {pct(lead)}; "
              f"exits stored before the consumer needed them in {(lead > 0).mean() * 100:.1f}%, "
              f"more than 2 us before in {(lead > 2).mean() * 100:.1f}%")
        # step periods: published(t, s) - published(t, s-1); the input of step s is
        # the hand-off of step s-1 (phase gs = s-1)
        okb = have[3][:, :, 1:] & have[3][:, :, :-1]
        per = us((br[:, :, 1:] - br[:, :, :-1]) % (1 << 32))
        wmask = np.zeros_like(okb)
        wfull = np.zeros(have[1].shape, bool)
        wfull[:, :-1, :] = ok & (us((hd[:, :-1, :] - nd[:, :-1, :]) % (1 << 32)) > 0.2)
        wmask[:, :, :] = wfull[:, :, :-1]
        print(f"    step (input hop waited) {pct(per[okb & wmask])}")
        print(f"    step (input was ready)  {pct(per[okb & ~wmask])}")
        okl = have[3][:, :-1, 1:] & have[3][:, 1:, :-1]
        lag = us((br[:, :-1, 1:] - br[:, 1:, :-1]) % (1 << 32))
        lag = np.where(lag > 2 ** 31 / 100, lag - 2 ** 32 / 100, lag)
        print(f"    lag behind the producer tile {pct(lag[okl])}")
        # producer wave 0: its step s-1 published -> its step s exit stores (d1)
        okd = have[0][:, :, 1:] & have[3][:, :, :-1]
        d1 = us((st[:, :, 1:] - br[:, :, :-1]) % (1 << 32))[okd]
        print(f"    d1 published(s-1) -> exit stores of s issued {pct(d1)}")
        # per tile: first and last barrier, steps; tiles in progress over time
        tb = np.where(have[3], us((br - t0) % (1 << 32)), np.nan)
        first = np.nanmin(tb, axis=2).ravel()
        last = np.nanmax(tb, axis=2).ravel()
        nst = have[3].sum(axis=2).ravel()
        ok_t = nst > 0
        first, last, nst = first[ok_t], last[ok_t], nst[ok_t]
        dur = last - first
        print(f"    tiles {ok_t.sum()}: steps {pct(nst.astype(float))}".replace(" us", ""))
        print(f"    tile duration {pct(dur)}; per-step period over a tile {pct(dur / np.maximum(nst - 1, 1))}")
        span = np.nanmax(last)
        cuts = np.linspace(0, span, 11)[:-1]
        act = [int(((first <= c) & (last >= c)).sum()) for c in cuts]
        print(f"    tiles in progress at 0..90% of the span: {act}")


if __name__ == "__main__":
    main()
