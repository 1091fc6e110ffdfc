"""Host checks of the light lattice (kLightsGridA10/A01): which light sets
light_grid_build accepts, and -- for accepted lattices -- that the kernel's
cell lookup (restated with the same float operations) never misses a light
the exact axis-aligned test hits, for random rays and for rays aimed at cell
edges and corners. The GPU half is tests/test_gpu_parity.py::test_light_grid_*."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from ipt_amd import scenes

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("lgrid") / "light_grid_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-DIPT_HD=inline", "-o", str(exe),
                    str(HERE / "native" / "light_grid_check.cpp")], check=True)
    return exe


def _run(exe, lights, rays=20000):
    lines = [str(len(lights))]
    for L in lights:
        vals = list(L["position"]) + list(L["x_axis"]) + list(L["y_axis"]) + [L["power"], L["type"]]
        lines.append(" ".join(repr(float(np.float32(v))) for v in vals))
    r = subprocess.run([str(exe), str(rays)], input="\n".join(lines) + "\n", capture_output=True, text=True)
    out = dict()
    for line in r.stdout.split("\n"):
        w = line.split()
        for i in range(0, len(w) - 1, 2):
            out[w[i]] = int(w[i + 1])
    return r.returncode, out


@pytest.mark.parametrize("k", [5, 8, 16, 32])
def test_lattice_accepted_and_lookup_complete(checker, k):
    rc, out = _run(checker, scenes.make_scene_box_lights(k)["lights"])
    assert rc == 0, out
    assert out["lattice"] == 1 and out["nu"] == k and out["nv"] == k
    assert out["hits"] > 0 and out["missed"] == 0


def test_lattice_with_empty_row(checker):
    L = scenes.make_scene_box_lights(8)["lights"]
    rc, out = _run(checker, L[:8] + L[16:])
    assert rc == 0 and out["lattice"] == 1 and out["missed"] == 0


@pytest.mark.parametrize("variant", ["nudged", "mixed_axes", "not_coplanar", "overlap", "random"])
def test_not_a_lattice(checker, variant):
    L = [dict(l) for l in scenes.make_scene_box_lights(8)["lights"]]
    if variant == "nudged":
        c = list(L[9]["position"])
        c[1] = float(np.float32(c[1] + np.float32(0.0025)))
        L[9]["position"] = c
    elif variant == "mixed_axes":
        L[3]["x_axis"], L[3]["y_axis"] = L[3]["y_axis"], L[3]["x_axis"]
    elif variant == "not_coplanar":
        c = list(L[5]["position"])
        c[2] = float(np.float32(c[2] - np.float32(0.01)))
        L[5]["position"] = c
    elif variant == "overlap":
        L.append(dict(L[0]))
    else:
        L = scenes.make_scene_random_lights(64, seed=7)["lights"]
    rc, out = _run(checker, L, rays=10)
    assert rc == 0 and out["lattice"] == 0
