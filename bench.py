#!/usr/bin/env python3
"""bench.py -- Mpixel-disparities/s of the MI355X semi-global matcher.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
it is launched once per GPU by torch.distributed.run.  One step = one pass of
the hot path over one stereo pair per GPU (pairs shard one per GPU, SURVEY.md
section 8e), inputs already resident in HBM, followed by the RCCL gather of
the disparity maps to rank 0 when N > 1.  Rank 0 prints ONE JSON line.

Metric (BASELINE.json): V*W*H*D / t in Mpixel-disparities/s, V = views
aggregated.  Default workload = BASELINE.json configs[1] ("config 2"):
1242x375, D=128, census 9x7 + 8-path SGM + WTA, left view (V=1).

roofline: the dominant kernel (largest share of the per-step kernel time),
its algorithmic bytes per launch (DESIGN.md "Roofline") over its average
launch duration, measured with HIP events recorded by libsgm_hip.so around
every launch on the stream that launch runs on (sgm_set_profiling), in a
second pass of the same K steps right after the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpixel-disparities/s, 8-path SGM @ KITTI 1242×375 D=128; 1→8 GPU scaling"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)

CONFIGS = {
    # BASELINE.json configs[0] ("config 1"): the reference's CPU-runnable case;
    # here both the GPU path and the CPU baseline run it
    "k64": dict(h=375, w=1242, D=64, views=2,
                workload="config1: KITTI 1242x375 D=64, both views + LR check (V=2), 1 pair per GPU"),
    "k128": dict(h=375, w=1242, D=128, views=1,
                 workload="config2: KITTI 1242x375 D=128, census 9x7 + Hamming cost + 8-path "
                          "SGM + WTA/uniqueness/sub-pixel, left view (V=1), 1 pair per GPU"),
    "k128lr": dict(h=375, w=1242, D=128, views=2,
                   workload="KITTI 1242x375 D=128, both views + LR check (V=2), 1 pair per GPU"),
    "hd256": dict(h=1080, w=1920, D=256, views=2,
                  workload="config3: 1920x1080 D=256, 8-path SGM + LR check (V=2), 1 pair per GPU"),
    "4k256": dict(h=2160, w=3840, D=256, views=2,
                  workload="3840x2160 D=256, 8-path SGM + LR check (V=2), 1 pair per GPU"),
    # BASELINE.json configs[4] on one GPU: the full pipeline of node.cpp:80-107
    "4k256full": dict(h=2160, w=3840, D=256, views=2, full=True,
                      workload="config5: 3840x2160 D=256 full pipeline: sky detector on both "
                               "views + 8-path SGM + LR check + post_filter + LKRefine (V=2), "
                               "1 pair per GPU"),
    "k128full": dict(h=375, w=1242, D=128, views=2, full=True,
                     workload="KITTI 1242x375 D=128 full pipeline: sky detector on both views + "
                              "8-path SGM + LR check + post_filter + LKRefine (V=2), 1 pair per GPU"),
}

# Algorithmic HBM bytes per pixel-disparity element per launch (DESIGN.md
# "Roofline"): f32 volumes, each read or written once; checkpoints are one
# D-vector per K steps (H/D2: K = 16, 8 at D = 256; V: K = 8, 4 at D = 256).
# regions the library times around launches that run concurrently -> those launches
CONCURRENT_REGIONS = {"slant_down_hpair": ("slant_down", "stage_a_h")}


def bytes_per_elem(name: str, D: int) -> float:
    ck = 4.0 / (8 if D >= 256 else 16)      # H and D2 families
    ckv = 4.0 / (4 if D >= 256 else 8)      # vertical family
    table = {
        "cost_h": 4.0,                  # write C_h (census rows come from LDS)
        "vfwd": 8.0 + ckv,              # read C_h, write C, write L3 checkpoints
        "pair_fwd_L1": 4.0 + ck, "pair_fwd_L3": 4.0 + ckv, "pair_fwd_L6": 4.0 + ck,
        "pair_bwd_L2_init2": 8.0 + ck,  # read C + ckpt, write S12
        "pair_bwd_L7_acc": 12.0 + ck,   # read C + T5 + ckpt, write T
        "pair_bwd_L4_final": 12.0 + ckv,  # read C + S12 + T + ckpt
        # multi-role launches (sums of their roles)
        "stage_a": (4.0 + ck) + 8.0 + (4.0 + ck),   # L1 fwd | L5 -> T5 | L6 fwd
        "stage_b": (8.0 + ck) + (12.0 + ck),        # L2 bwd -> S12 | L7 bwd -> T
        # the banded schedule (volumes above the Infinity Cache): stage A also
        # runs L2 bwd -> S12, stage B's bands only L7 bwd -> T
        "stage_a_hp": (4.0 + ck) + 8.0 + (4.0 + ck) + (8.0 + ck),
        "stage_b_d2": 12.0 + ck,
        # the forward bands: stage A's diagonal roles per band (L5 -> T5 |
        # L6 fwd), then the whole H pair as its own launch
        "stage_a_d": 8.0 + (4.0 + ck),
        "stage_a_h": (4.0 + ck) + (8.0 + ck),
        # the slanted-tile schedule (DESIGN.md "Slanted tiles"): vfwd writing
        # the whole L3 volume; the top-down pass reads C and writes T56; the
        # bottom-up pass reads C, S12, L3 and T56.  Each tile (NW = 14 columns
        # top-down, 15 bottom-up) also hands 2 (top-down) or 3 (bottom-up)
        # D-vectors per step to the next tile as 8-byte granules, written
        # once and read once
        "vfwd_l3": 12.0,
        # its cost stage as checkpoints + strips (sgm_vstrip.hip):
        # the horizontal IIR's state (3 floats) at every 16-column strip edge,
        # written by cost_ck and read by vstrip, which writes C and L3
        "cost_ck": 3 * 4.0 / 16,
        "vstrip": 3 * 4.0 / 16 + 8.0,
        "slant_down": 8.0 + 2 * 16.0 / 14,
        "slant_up": 16.0 + 3 * 16.0 / 15,
    }
    # the top-down pass and the H pair run concurrently (two streams); the
    # library also times the pair as one region, fork to join
    table["slant_down_hpair"] = table["slant_down"] + table["stage_a_h"]
    if name in table:
        return table[name]
    if name.startswith("sweep_"):
        return {"init": 8.0, "acc": 12.0, "final": 12.0, "store": 8.0}[name.rsplit("_", 1)[1]]
    return 0.0


# Of those bytes, the reads of the final cost volume C (4 B per element per
# path direction that walks it).  At K128/K64 C (238.5 / 119 MB) stays in the
# 256 MB Infinity Cache through the aggregation (DESIGN.md "Infinity Cache"),
# so algorithmic bytes minus these are the bytes the kernel moves to/from HBM.
def c_read_bytes_per_elem(name: str) -> float:
    table = {"stage_a": 12.0, "stage_b": 8.0, "pair_bwd_L4_final": 4.0, "sweep_L8_acc": 4.0,
             "stage_a_hp": 16.0, "stage_b_d2": 4.0, "stage_a_d": 8.0, "stage_a_h": 8.0,
             "pair_fwd_L1": 4.0, "pair_fwd_L3": 4.0, "pair_fwd_L6": 4.0,
             "pair_bwd_L2_init2": 4.0, "pair_bwd_L7_acc": 4.0, "slant_down": 4.0, "slant_up": 4.0,
             "slant_down_hpair": 12.0}
    if name in table:
        return table[name]
    return 4.0 if name.startswith("sweep_") else 0.0


def source_sha() -> str:
    """sha256 (first 16 hex digits) over the library's sources: ties a PMC
    traffic record (profiles/pmc_traffic.json) to the code it was taken on."""
    import hashlib
    csrc = os.path.join(ROOT, "stereo_matching_amd", "csrc")
    hsh = hashlib.sha256()
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")) or f == "Makefile":
            with open(os.path.join(csrc, f), "rb") as fh:
                hsh.update(f.encode() + b"\0" + fh.read())
    return hsh.hexdigest()[:16]


BYTES_PER_PIXEL = {"census": 9, "lr": 12,
                   # post_filter (sgm_post.hip), per pixel and launch: the fill reads
                   # the original and working maps (8); labelling reads the map and
                   # writes label + count (12); the area test reads map, 2 labels,
                   # area and writes the map (16); count/merge touch few pixels
                   "post_prep": 12, "post_median": 8, "post_cc_local": 16, "post_cc_apply": 20,
                   "post_cc_count": 4, "post_cc_merge": 0,
                   # LKRefine: map in + out, 7x7 window and images through LDS/L2
                   "lk_refine": 10,
                   # sky detector: image in, gray out/in, mask out (+ per-threshold columns)
                   "sky_detect": 4, "bm_wta": 0}


def algorithmic_bytes(name: str, elems: float, D: int) -> float:
    if name == "bm_wta":
        return 4.0 * elems  # read the filtered cost once (elems = W*H*D)
    if name in BYTES_PER_PIXEL:
        # per-pixel classes report elems = pixels (census: W*H; post_*: W*H)
        return BYTES_PER_PIXEL[name] * elems
    return bytes_per_elem(name, D) * elems


def cpu_model() -> str:
    """The host CPU's model name (SURVEY.md 8d asks for it beside the baseline)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="k128", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=3,
                    help="minimum samples of the CPU baseline (median reported); sampling goes on "
                         "until --cpu-seconds of CPU work have run (at most 12 samples)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU work the baseline sample spans (the contract asks for ~10-30 s)")
    ap.add_argument("--no-profile-pass", action="store_true")
    ap.add_argument("--post-filter", action="store_true",
                    help="end each step with post_filter() on the GPU (SGM.cpp:821; V=2 configs)")
    ap.add_argument("--lk-refine", action="store_true",
                    help="end each step with LKRefine on the GPU (SGM.cpp:824, LKSubPixelImpl.cpp)")
    ap.add_argument("--sky-detect", action="store_true",
                    help="start each step with the sky detector on both views (node.cpp:80-93)")
    # 4: one collective per 4 steps' maps measured 1.9% faster per step than one per step
    # under torchrun at world 1 (profiles/r03_experiments/gather_batching.txt); the
    # last batch's gather runs after the last step (~50 us at N = 8 per timed region)
    ap.add_argument("--gather-every", type=int, default=4,
                    help="N > 1: gather the maps of this many steps in one collective")
    ap.add_argument("--no-gather", action="store_true",
                    help="diagnostic: N > 1 without the gather of the maps (not a valid bench line)")
    ap.add_argument("--caller-stream", action="store_true",
                    help="diagnostic: run the frames on a stream of the caller's instead of the "
                         "handle's own (each call then records an event as it returns)")
    ap.add_argument("--graph", action="store_true",
                    help="single process: time replays of one frame captured as a HIP graph "
                         "(the per-kernel profile pass still runs eagerly)")
    ap.add_argument("--view-split", action="store_true",
                    help="N even, V=2 configs: one pair per two GPUs, left view on the even rank, "
                         "right view on the odd one, F_R over RCCL point-to-point (SURVEY.md 8e "
                         "optional split; a latency option, not the default sharding)")
    ap.add_argument("--host-io", action="store_true",
                    help="also time sgm_process on host buffers (PCIe-inclusive, not `value`)")
    return ap.parse_args()


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    h, w, D, views = cfg["h"], cfg["w"], cfg["D"], cfg["views"]

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a SCALE line must describe the ranks that ran: refuse a mismatch
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world} (launch N ranks "
                         f"with --gpus N)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # under torch.distributed.run (the driver's launch line for N > 1, and the
    # GPU test of that line at N = 1) the process group comes up on RCCL
    distributed = world > 1 or "LOCAL_WORLD_SIZE" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=dev)
    if args.view_split and (world % 2 or views != 2):
        raise SystemExit("--view-split needs an even number of ranks and a two-view config")

    from stereo_matching_amd import SGM, synthetic

    # one synthetic pair per rank (weak scaling: per-GPU work is fixed); with
    # --view-split one pair per two ranks
    left, right = synthetic.stereo_pair(h, w, D, pair_index=rank // 2 if args.view_split else rank)
    d_left = torch.from_numpy(left).to(dev)
    d_right = torch.from_numpy(right).to(dev)
    d_out = torch.empty((h, w), dtype=torch.float32, device=dev)
    # N > 1: each step's map goes to rank 0 by a gather that overlaps the next
    # step's kernels (double-buffered maps, stereo_matching_amd.distributed)
    pipe = None
    gk = max(1, args.gather_every)
    if distributed and not args.view_split and not args.no_gather:
        from stereo_matching_amd.distributed import PipelinedGather
        pipe = PipelinedGather((gk, h, w) if gk > 1 else (h, w), torch.float32, dev, depth=2)
    nstep = [0]
    verified = []

    if cfg.get("full"):
        args.post_filter = args.lk_refine = args.sky_detect = True
    team = None
    if args.view_split:
        from stereo_matching_amd.distributed import ViewSplit
        sgm = SGM(h, w, 1, D, views=1, view="right" if rank % 2 else "left", device=local,
                  sky_detect=args.sky_detect)
        team = ViewSplit(sgm, h, w, dev, post_filter=args.post_filter, lk_refine=args.lk_refine)
    else:
        sgm = SGM(h, w, 1, D, views=views, device=local, post_filter=args.post_filter,
                  lk_refine=args.lk_refine, sky_detect=args.sky_detect)
    # one stream for everything a step enqueues (the library's kernels,
    # torch's copies, RCCL's stream dependencies): the handle's own stream
    # (sgm_get_stream), so the library's calls record no events (a call on a
    # caller's stream records one as it returns: a ~5 us gap before the next
    # frame's first kernel)
    torch.cuda.synchronize(dev)
    stream = (torch.cuda.Stream(dev) if args.caller_stream
              else torch.cuda.ExternalStream(sgm.stream, device=dev))
    torch.cuda.set_stream(stream)
    if pipe:
        pipe.check = sgm.check

    def verify(what):
        """After a pass: sgm_check on every rank (waits for the frames; raises
        if a slanted-pass hand-off gave up in one), agreed across ranks, so
        no invalid frame is timed or gathered as valid; exits non-zero."""
        try:
            if pipe:
                pipe.verify()
            else:
                err = None
                try:
                    sgm.check()
                except Exception as e:  # noqa: BLE001 -- agreed on below
                    err = e
                if distributed:
                    from stereo_matching_amd.distributed import agree
                    if not agree(err is None) and err is None:
                        err = RuntimeError("a frame on another rank is invalid")
                if err is not None:
                    raise err
        except Exception as e:  # noqa: BLE001
            print(f"bench.py: the {what} pass produced invalid frames: {e}", file=sys.stderr)
            sys.exit(3)
        verified.append(what)

    def step():
        if team:
            team.step(d_left.data_ptr(), d_right.data_ptr(), d_out)
            return
        out = d_out
        if pipe:
            out = pipe.buffer()
            out = out[nstep[0] % gk] if gk > 1 else out
        sgm.process_device(d_left.data_ptr(), d_right.data_ptr(), out.data_ptr(),
                           stream=stream.cuda_stream)
        nstep[0] += 1
        if pipe and nstep[0] % gk == 0:
            pipe.submit()

    def flush():  # a partial batch of maps goes out before a drain
        if pipe and nstep[0] % gk:
            pipe.submit()
        nstep[0] = 0

    for _ in range(args.warmup):
        step()
    flush()
    if pipe:
        pipe.drain(verify=False)
    torch.cuda.synchronize(dev)
    verify("warmup")
    eager_step = step
    if args.graph:
        # the frame's launches recorded once on the handle's stream (no event
        # records there, so the whole frame is capturable) and replayed as one
        # graph launch per step
        if pipe or team:
            raise SystemExit("--graph: single-process runs only")
        if args.post_filter:
            # the median fill's launch count is read back to the host each
            # round; the library refuses to capture it (sgm_capi.hip post_filter)
            raise SystemExit("--graph: not with post_filter (full configs); its launch count is "
                             "decided on the host")
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
            eager_step()
        torch.cuda.synchronize(dev)

        def step():
            graph.replay()

    def timed_steps(k):
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        flush()
        if pipe:
            pipe.drain(verify=False)  # every gather of the timed steps is inside the timed region
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        return time.perf_counter() - t0

    elapsed = timed_steps(args.steps)
    verify("timed")
    rank_min = rank_max = elapsed
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rank_max = elapsed = float(t.item())
        t = torch.tensor([rank_min], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        rank_min = float(t.item())

    pairs = world // 2 if args.view_split else world
    units = float(pairs) * views * h * w * D * args.steps
    value = units / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # per-kernel durations: HIP events around every launch, same K steps
    roofline = None
    kernels = {}
    if not args.no_profile_pass:
        sgm.set_profiling(True)
        step = eager_step
        prof_elapsed = timed_steps(args.steps)
        verify("profile")
        prof = sgm.get_profile()
        sgm.set_profiling(False)
        for name, (n, total_ms, elems) in prof.items():
            kernels[name] = dict(launches=n, avg_us=round(total_ms / n * 1e3, 2),
                                 share_per_step_ms=round(total_ms / args.steps, 4),
                                 algo_bytes=algorithmic_bytes(name, elems, D))
        # launches that ran concurrently inside a region the library also
        # times as a whole (the slanted schedule's top-down pass beside the H
        # pair): the region stands for them in the kernel sum and the
        # aggregation set, and gets its own block (`concurrent_region`); the
        # dominant KERNEL is the longest launch that ran alone (a concurrent
        # launch's duration is shared time, and tracing tools time it
        # differently: rocprofv3's kernel trace stretched the pair by up to 14%
        # on one box)
        concurrent = {}
        for region, parts in CONCURRENT_REGIONS.items():
            if region in kernels:
                for k in parts:
                    if k in kernels:
                        kernels[k]["concurrent_in"] = region
                        concurrent[k] = region
        solo = [k for k in kernels if k not in concurrent]
        alone = [k for k in solo if k not in CONCURRENT_REGIONS]
        if kernels:
            dom = max(alone or solo, key=lambda k: kernels[k]["share_per_step_ms"])
            kd = kernels[dom]
            achieved = kd["algo_bytes"] / (kd["avg_us"] * 1e-6) / 1e9
            traffic = None
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                try:
                    with open(pmc) as fh:
                        rec = json.load(fh).get(args.config, {})
                    traffic = rec.get(dom)
                    if traffic is None and dom in CONCURRENT_REGIONS and \
                            all(p in rec for p in CONCURRENT_REGIONS[dom]):
                        traffic = sum(rec[p] for p in CONCURRENT_REGIONS[dom])
                except (OSError, ValueError):
                    traffic = None
            tag = pmc_tag = None
            src = source_sha()
            if traffic is not None:
                with open(pmc) as fh:
                    pmc_tag = json.load(fh).get("_tags", {}).get(args.config)
                tag = pmc_tag.get("tag") if isinstance(pmc_tag, dict) else pmc_tag
            # streams only: without the reads of C, which the Infinity Cache
            # serves when the volume fits it (K64/K128); above it they are HBM
            # reads too and frac is already the HBM figure
            fits = h * w * D * 4 <= (256 << 20)
            cbytes = c_read_bytes_per_elem(dom) * kd["algo_bytes"] / max(bytes_per_elem(dom, D), 1e-9) \
                if fits and bytes_per_elem(dom, D) else 0.0
            streams = (kd["algo_bytes"] - cbytes) / (kd["avg_us"] * 1e-6) / 1e9
            kernel_sum_ms = sum(kernels[k]["share_per_step_ms"] for k in solo)
            # `achieved` / `frac`: the dominant kernel's algorithmic bytes that
            # travel to or from HBM, over its launch time.  When the cost
            # volume fits the 256 MB Infinity Cache (K64/K128) its reads of C
            # are served on-die and are left out; above it every algorithmic
            # byte is an HBM byte.  The algorithmic rate including those reads
            # is `achieved_algorithmic` / `frac_algorithmic` (a memory-side
            # rate, not an HBM one).  `traffic` is the PMC memory-side count
            # (FETCH_SIZE x 2 + WRITE_SIZE, Infinity-Cache hits included).
            roofline = {"bound": "hbm", "kernel": dom, "achieved": round(streams, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(streams / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_scope": "memory-side bytes per launch (PMC), Infinity-Cache hits "
                                         "included",
                        "traffic_tag": tag,
                        "traffic_src_sha": pmc_tag.get("src_sha") if isinstance(pmc_tag, dict) else None,
                        "src_sha": src,
                        "traffic_matches_source": bool(isinstance(pmc_tag, dict)
                                                       and pmc_tag.get("src_sha") == src),
                        "algo_bytes_per_launch": kd["algo_bytes"],
                        "hbm_algo_bytes_per_launch": kd["algo_bytes"] - cbytes,
                        "avg_launch_us": kd["avg_us"],
                        "c_cache_resident": fits,
                        "achieved_algorithmic": round(achieved, 1),
                        "frac_algorithmic": round(achieved / HBM_PEAK_GBS, 4),
                        # per-kernel times come from a second, event-bracketed pass;
                        # flag when its kernel sum exceeds the timed step
                        "kernel_sum_ms_per_step": round(kernel_sum_ms, 4),
                        "profile_pass_ms_per_step": round(prof_elapsed / args.steps * 1e3, 4),
                        "kernel_sum_exceeds_timed_step": kernel_sum_ms > ms_per_step}
            for region, parts in CONCURRENT_REGIONS.items():
                if region not in kernels:
                    continue
                kr = kernels[region]
                rate = kr["algo_bytes"] / (kr["avg_us"] * 1e-6) / 1e9
                rtraffic = None
                try:
                    with open(pmc) as fh:
                        rec = json.load(fh).get(args.config, {})
                    if all(p in rec for p in parts):
                        rtraffic = sum(rec[p] for p in parts)
                except (OSError, ValueError):
                    rtraffic = None
                roofline["concurrent_region"] = {
                    "name": region, "kernels": list(parts), "bound": "hbm",
                    "wall_us": kr["avg_us"], "share_per_step_ms": kr["share_per_step_ms"],
                    "algo_bytes_per_launch": kr["algo_bytes"], "achieved": round(rate, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(rate / HBM_PEAK_GBS, 4),
                    "traffic": rtraffic,
                    "scope": "fork to join on the frame's stream (HIP events); its kernels run "
                             "at the same time on two streams"}
            # the 8-path aggregation kernels (everything after the cost volume
            # except vfwd, which is mostly the vertical cost filter)
            agg = [k for k in solo if k.startswith(("sweep_", "pair_", "stage_", "slant_"))]
            post = [k for k in kernels if k.startswith("post_")]
            if post:
                roofline["post_filter_ms_per_step"] = round(
                    sum(kernels[k]["share_per_step_ms"] for k in post), 4)
            agg_ms = sum(kernels[k]["share_per_step_ms"] for k in agg)
            if agg_ms > 0:
                agg_bytes = sum(kernels[k]["algo_bytes"] * kernels[k]["launches"] / args.steps
                                for k in agg)
                agg_c = sum(c_read_bytes_per_elem(k) / max(bytes_per_elem(k, D), 1e-9)
                            * kernels[k]["algo_bytes"] * kernels[k]["launches"] / args.steps
                            for k in agg if bytes_per_elem(k, D)) if fits else 0.0
                roofline["aggregation_set"] = {
                    "kernels": sorted(agg),
                    "algo_bytes_per_step": agg_bytes,
                    "hbm_algo_bytes_per_step": agg_bytes - agg_c,
                    "kernel_ms_per_step": round(agg_ms, 4),
                    "achieved": round((agg_bytes - agg_c) / (agg_ms * 1e-3) / 1e9, 1),
                    "frac": round((agg_bytes - agg_c) / (agg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "achieved_algorithmic": round(agg_bytes / (agg_ms * 1e-3) / 1e9, 1),
                    "frac_algorithmic": round(agg_bytes / (agg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "bytes_per_elem_per_view": round(agg_bytes / (views * h * w * D), 2)}

    host_io = None
    if args.host_io and rank == 0:
        # PCIe-inclusive rate: host images in, host disparity out (sgm_process)
        ts = []
        for _ in range(max(3, args.steps)):
            t0 = time.perf_counter()
            sgm.process(left, right)
            ts.append(time.perf_counter() - t0)
        th = statistics.median(ts)
        host_io = {"value": round(views * h * w * D / th / 1e6, 1), "unit": "Mpixel-disparities/s",
                   "ms_per_frame": round(th * 1e3, 4),
                   "scope": "sgm_process: H2D images, pipeline, D2H disparity, synchronous"}

    cpu = None
    cpu_note = None
    if world > 1:
        cpu_note = ("measured on rank 0 at N=1 only (bench contract); the N=1 line of the same "
                    "config carries it")
    elif rank == 0 and not args.no_cpu_baseline:
        import oracle
        oracle.build()
        # every host thread this process may use: OMP_NUM_THREADS when the
        # environment sets it (the GPU pool sets it to the box's CPU share),
        # else all host CPUs
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
        oracle.set_threads(threads)
        # bounded sample (~0.6 G pixel-disparity units per frame): a band of the
        # frame's top rows at full width when the frame is larger than that
        sh = h if views * h * w * D <= 6e8 else max(16, int(6e8 / (views * w * D)))
        ls, rs = left[:sh], right[:sh]
        full = bool(cfg.get("full"))
        ts = []
        while len(ts) < max(1, args.cpu_frames) or (sum(ts) < args.cpu_seconds and len(ts) < 12):
            t0 = time.perf_counter()
            ml = oracle.sky_detect(ls) if full else None
            mr = oracle.sky_detect(rs) if full else None
            ref = oracle.process(ls, rs, D, views=views, sky_l=ml, sky_r=mr, schedule="refplace")
            if full:
                oracle.lk_refine(ls, rs, ref["final"], D)
            ts.append(time.perf_counter() - t0)
        tmed = statistics.median(ts)
        what = "full frames" if sh == h else f"bands of the top {sh} rows (full width)"
        stages = ("sky detector + SGM + LR + post_filter + LKRefine" if full else
                  "SGM" + (" + LR + post_filter" if views == 2 else ""))
        try:
            affinity = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            affinity = None
        cpu = {"value": round(views * sh * w * D / tmed / 1e6, 2), "unit": "Mpixel-disparities/s",
               "cores": oracle.max_threads(), "kind": "port", "placement": "reference",
               "omp_max_threads": oracle.max_threads(), "host_cpus": os.cpu_count(),
               "affinity_cpus": affinity, "cpu_model": cpu_model(),
               "sample": f"{len(ts)} {what} of the same workload ({w}x{h} D={D}, V={views}; "
                         f"{stages}) through orc_process_refplace (oracle/sgm_oracle.c): the "
                         f"reference's loop nests and OpenMP placement -- parallel only at its "
                         f"`omp parallel for` sites, both cost filters and the aggregation + WTA "
                         f"sequential, 10 volumes -- median {tmed:.3f} s per sample"}

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mpixel-disparities/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "pairs_per_s": round(pairs * args.steps / elapsed, 2),
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": cfg["workload"] if cfg.get("full") else
                       cfg["workload"] + (" + sky detector" if args.sky_detect else "")
                       + (" + post_filter" if args.post_filter else "")
                       + (" + LKRefine" if args.lk_refine else ""),
                       "width": w, "height": h, "max_disp": D, "views": views,
                       "post_filter": bool(args.post_filter), "lk_refine": bool(args.lk_refine),
                       "sky_detect": bool(args.sky_detect),
                       "launch": "one HIP graph replay per frame" if args.graph else "eager",
                       "pairs_per_gpu": 0.5 if args.view_split else 1, "global_batch": pairs,
                       "parallelism": (f"view-split x{pairs} (left/right view per GPU, F_R over "
                                       f"RCCL point-to-point; maps stay on the even ranks)"
                                       if args.view_split else
                                       (f"pair-sharded x{world} (1 pair/GPU), NO gather (diagnostic)"
                                        if args.no_gather else
                                        f"pair-sharded x{world} (1 pair/GPU), RCCL gather to rank 0 "
                                        + (f"of every {gk} steps' maps in one collective, "
                                           if gk > 1 else "")
                                        + ("overlapped with the following steps" if gk > 1
                                           else "overlapped with the next step")) if distributed else
                                       "1 pair on 1 GPU (single process: no process group, no "
                                       "gather)")},
            # what the process group saw (the driver's SCALE runs check it
            # against n_gpus), and the spread of the timed region over ranks
            "backend": dist.get_backend() if distributed else None,
            "world_size_seen": dist.get_world_size() if distributed else 1,
            "rank_timed_s": {"min": round(rank_min, 6), "max": round(rank_max, 6)},
            # passes whose frames sgm_check found valid on every rank
            "frames_verified": verified,
            "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels,
            **({"cpu_baseline_note": cpu_note} if cpu_note else {}),
            "host_io": host_io,
        }
        print(json.dumps(rec))
    sgm.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
