"""CPU checks of bench.py's bookkeeping (no GPU): the algorithmic-byte tables
agree with DESIGN.md's schedule, the HBM-only view never exceeds the
algorithmic one, and the source hash that ties profiles/pmc_traffic.json to
the code is stable and covers every library source."""
from __future__ import annotations

import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("D", [32, 64, 128, 256])
def test_schedule_bytes(D):
    # 74 B/elem per view at D <= 128 for cost + aggregation
    # (cost_h 4 + vfwd 8.5 + stage A 16.5 + stage B 20.5 + L8 12 + final 12.5)
    total = sum(bench.bytes_per_elem(k, D) for k in
                ("cost_h", "vfwd", "stage_a", "stage_b", "sweep_L8_acc", "pair_bwd_L4_final"))
    ck = 4.0 / (8 if D >= 256 else 16)
    ckv = 4.0 / (4 if D >= 256 else 8)
    assert total == pytest.approx(4 + (8 + ckv) + (16 + 2 * ck) + (20 + 2 * ck) + 12 + (12 + ckv))
    if D <= 128:
        assert total == pytest.approx(74.0)


def test_c_reads_within_algorithmic_bytes():
    for k in ("stage_a", "stage_b", "pair_bwd_L4_final", "sweep_L8_acc", "stage_a_hp",
              "stage_b_d2", "stage_a_d", "stage_a_h"):
        for D in (64, 128, 256):
            assert 0 < bench.c_read_bytes_per_elem(k) < bench.bytes_per_elem(k, D), (k, D)
    assert bench.c_read_bytes_per_elem("cost_h") == 0 and bench.c_read_bytes_per_elem("vfwd") == 0


def test_source_sha_stable_and_complete():
    a, b = bench.source_sha(), bench.source_sha()
    assert a == b and len(a) == 16
    # the PMC records name the source hash they were taken on
    pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    for cfg in ("k128", "k128lr", "hd256", "4k256"):
        tag = pmc["_tags"][cfg]
        assert isinstance(tag, dict) and tag["src_sha"] and tag["git"], cfg


def test_configs_cover_baseline():
    # BASELINE.json configs: K64 (config 1), K128 V=1 (2), HD256 V=2 (3), 4K256 full (5)
    c = bench.CONFIGS
    assert (c["k64"]["D"], c["k64"]["views"]) == (64, 2)
    assert (c["k128"]["D"], c["k128"]["views"]) == (128, 1)
    assert (c["hd256"]["h"], c["hd256"]["w"], c["hd256"]["views"]) == (1080, 1920, 2)
    assert c["4k256full"].get("full") and c["4k256full"]["D"] == 256


def test_gpus_must_match_world_size():
    # a bench line must describe the ranks that ran: --gpus N without N ranks
    # exits non-zero before touching a GPU (no WORLD_SIZE = one rank)
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE 1" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


# kernel families the frame schedules launch (sgm_capi.hip run_frame): every
# instantiation the library holds must map to a profiler name, so that the PMC
# passes (tools/pmc_reduce.py) and the timer check see each launch of a frame
FRAME_KERNELS = ("census_kernel<", "cost_h_kernel<", "cost_h2_kernel<", "cost_h_global_kernel<",
                 "vfwd_kernel<", "vfwd2_kernel<", "stage_a_kernel<", "stage_a2_kernel<", "stage_b_kernel<",
                 "stage_b2_kernel<", "hpair_kernel<", "sweep_kernel<7", "sweep2_kernel<7",
                 "sweep_split_kernel<7", "pair_final_kernel<", "pair_final2_kernel<", "slant_kernel<",
                 "lr_kernel(", "lr_cm_kernel(", "lk_refine_kernel(", "median_fill_kernel<",
                 "cost_ck_kernel<", "vstrip_kernel<")


def test_pmc_reducer_names_every_frame_kernel():
    import shutil
    import subprocess
    import sys
    lib = os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip.so")
    if not os.path.exists(lib) or not shutil.which("nm"):
        pytest.skip("library not built or no nm")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_reduce import short
    out = subprocess.run(["nm", "-C", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    names = {ln.split(" ", 2)[2] for ln in out.splitlines() if ln.count(" ") >= 2 and "_kernel" in ln}
    seen = set()
    for fam in FRAME_KERNELS:
        inst = [n for n in names if "sgm::" + fam in n or "sgm::(anonymous namespace)::" + fam in n]
        assert inst, f"no {fam} in the library"
        for n in inst:
            assert short(n), f"tools/pmc_reduce.py cannot name {n}"
            seen.add(short(n))
    # the volume kernels among them carry algorithmic bytes in bench.py
    for k in ("cost_h", "vfwd", "vfwd_l3", "stage_a", "stage_b", "sweep_L8_acc", "pair_bwd_L4_final",
              "slant_down", "slant_up", "stage_a_h", "cost_ck", "vstrip"):
        assert k in seen and bench.bytes_per_elem(k, 128) > 0, k
