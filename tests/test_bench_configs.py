"""bench.py's workloads against BASELINE.json's configs (CPU only).

Each bench config must render the resolution and bounce depth its BASELINE
string names, and no more passes per step than the frame it is quoted on;
c3's two default steps are exactly its 64-spp frame.
"""
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

BASELINE = json.loads((ROOT / "BASELINE.json").read_text())["configs"]
INDEX = {"c1": 0, "c2": 1, "c3": 2, "c4": 3, "c5": 4}


def _parse(text):
    w, h = map(int, re.search(r"(\d+)x(\d+)", text).groups())
    spp = int(re.search(r"(\d+) spp", text).group(1))
    m = re.search(r"(\d+) bounces", text)
    return w, h, spp, int(m.group(1)) if m else None


def test_every_baseline_config_has_a_bench_workload():
    assert sorted(bench.CONFIGS) == sorted(INDEX)
    assert len(BASELINE) == len(INDEX)


def test_bench_workloads_match_baseline():
    for name, i in INDEX.items():
        scene, w, h, spp_step, steps, depth, scaling, _ = bench.CONFIGS[name]
        bw, bh, bspp, bdepth = _parse(BASELINE[i])
        assert (w, h) == (bw, bh), name
        if bdepth is not None:
            assert depth == bdepth, name
        assert spp_step <= bspp and bspp % spp_step == 0, name
        assert scaling in ("weak", "strong")


def test_c3_default_run_is_the_whole_frame():
    _, _, _, spp_step, steps, _, _, _ = bench.CONFIGS["c3"]
    assert spp_step * steps == _parse(BASELINE[2])[2]


def test_cpu_baseline_reports_threads_and_single_thread_rate():
    """The CPU-baseline leg (the oracle, test infrastructure) states the
    threads it used, the host's physical cores, a measured single-thread rate
    and the full-host extrapolation beside the measured figure (CPU only,
    a sub-second sample)."""
    import types

    a = types.SimpleNamespace(width=64, height=64, cpu_threads=2, cpu_sample=(16, 4), spp_per_step=1, steps=1,
                              n_rays=4, depth_max=3, seed=20241223, cpu_seconds=0.3)
    r = bench.cpu_baseline(a, bench.make_desc("box"))
    assert r["cores"] == 2 and r["value"] > 0 and r["kind"] == "port"
    assert r["single_thread_paths_per_s"] > 0 and r["thread_scaling"] > 0
    phys = bench.physical_cores()
    assert r["host_physical_cores"] == phys
    if phys:
        assert abs(r["full_host_extrapolated_Mpaths_s"] - r["single_thread_paths_per_s"] * phys / 1e6) < 1e-9


def test_oracle_sample_renderer_is_thread_invariant():
    """The CPU baseline's sampled renderer (one path per work item) gives the
    full renderer's values at the sampled pixels, for any thread count."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import oracle_binding as ob
    from ipt_amd import capi, scenes

    desc = scenes.make_scene_box()
    p = capi.make_params(48, 40, 2, n_rays=4, depth_max=3, seed=7)
    full, _ = ob.render_values(desc, p, n_threads=4)
    ref = None
    for th in (1, 3, 8):
        v, rows, cols = ob.render_rows_values(desc, p, 7, 2, 5, 1, n_threads=th)
        assert np.array_equal(v.view(np.uint32), full[:, rows][:, :, cols].view(np.uint32)), th
        ref = v if ref is None else ref
        assert np.array_equal(v.view(np.uint32), ref.view(np.uint32))
