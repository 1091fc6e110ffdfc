"""Statistical pinning of the estimator restatement against the survey's
measurements of the REAL reference (box scene,
640^2, 1 spp, n_rays 16, drand48 RNG). Our RNG differs, so agreement is
within Monte-Carlo error; tolerances are >= 3 sigma at these sizes."""
import pytest

import oracle_binding as ob
from ipt_amd import capi, scenes

# Appendix C, d=8 (== d>=6) and d=4 columns
REF_D8 = {"traced_rays": 165.5, "surface_hits": 104.7, "light_hits": 59.6,
          "expanded_nodes": 98.7, "iterations": 209.9, "light_samples": 105.0,
          "skipped": 45.4, "light_traces": 329.9}
REF_D4 = {"traced_rays": 92.0, "surface_hits": 58.0, "light_hits": 32.8, "expanded_nodes": 53.9}
REF_MEAN = {4: 0.06535, 5: 0.07358, 8: 0.08007}  # §6 table, "image mean"


@pytest.fixture(scope="module")
def runs(oracle):
    out = {}
    for d in (4, 5, 8):
        v, c, cnt = ob.render_values(scenes.make_scene_box(), capi.make_params(256, 256, 1, depth_max=d),
                                     0, with_counters=True)
        out[d] = (float(v.mean()), {k: x / cnt["paths"] for k, x in cnt.items()})
    return out


def test_event_counts_d8(runs):
    _, ev = runs[8]
    for k, ref in REF_D8.items():
        assert abs(ev[k] - ref) / ref < 0.03, (k, ev[k], ref)


def test_event_counts_d4(runs):
    _, ev = runs[4]
    for k, ref in REF_D4.items():
        assert abs(ev[k] - ref) / ref < 0.03, (k, ev[k], ref)


def test_image_means(runs):
    for d, ref in REF_MEAN.items():
        assert abs(runs[d][0] - ref) / ref < 0.04, (d, runs[d][0], ref)
    assert runs[4][0] < runs[5][0] < runs[8][0]


def test_depth_6_equals_8(oracle):
    """n_rays=16 reaches n=0 at depth 5, so depth_max 6 and 8 give identical
    images (verified on the reference)."""
    desc = scenes.make_scene_box()
    a, _ = ob.render_values(desc, capi.make_params(48, 48, 2, depth_max=6))
    b, _ = ob.render_values(desc, capi.make_params(48, 48, 2, depth_max=8))
    c, _ = ob.render_values(desc, capi.make_params(48, 48, 2, depth_max=5))
    assert (a.view("u4") == b.view("u4")).all()
    assert not (a.view("u4") == c.view("u4")).all()
