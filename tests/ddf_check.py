"""The reference's DDF chi^2 harness (test/check_ddf.cpp:11-203) restated,
vectorised: value_fn maps an (n, 3) array of directions to n values.

check_ddf(samples, value_fn): samples are the sampler's raw outputs in order;
vec3() outputs are retried as in check_ddf.cpp:90-96 (counted in total_tries),
the first N non-zero ones are bucketed over (alpha, phi), and chi^2 against
value * bucket area * N is accepted in [70, 135] * DoF/100 (check_ddf.cpp:
190-200). The DDF integral is the Monte-Carlo estimate of check_ddf.cpp:
29-70 (uniform sphere samples, value / (1/4pi)); the acceptance ratio N /
total_tries must match it (a sampler that returns vec3() with probability p
has a value function integrating to 1 - p)."""
import math

import numpy as np


def check_ddf(samples, value_fn, N=100000, size_alpha=20, size_phi=20, strict_integral=True, seed=7,
              sub=1):
    """sub > 1 integrates each bucket's expected count over sub x sub points
    (area-weighted) instead of the reference's value-at-centre x area: needed
    for DDFs that change inside one bucket, such as a light subtending a
    bucket or less; sub = 1 is check_ddf.cpp's rule."""
    samples = np.asarray(samples, np.float64)
    nz = np.any(samples != 0.0, axis=1)
    idx = np.nonzero(nz)[0]
    assert len(idx) >= N, ("not enough non-zero samples", len(idx), N)
    total_tries = int(idx[N - 1]) + 1
    v = samples[idx[:N]]
    rng = np.random.default_rng(seed)
    u1 = rng.random(200000) * 2 - 1
    u2 = rng.random(200000)
    r = np.sqrt(1 - u1 * u1)
    sph = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2), u1], 1).astype(np.float32)
    ddf_integral = float(np.mean(np.asarray(value_fn(sph), np.float64) / (0.25 / np.pi)))

    alpha = np.arccos(np.clip(v[:, 2], -1.0, 1.0))
    rr = np.hypot(v[:, 0], v[:, 1])
    s = np.clip(np.divide(v[:, 1], rr, out=np.zeros_like(rr), where=rr > 0), -1.0, 1.0)
    phi = np.where(v[:, 0] >= 0, np.arcsin(s), np.pi - np.arcsin(s))
    phi = np.where(phi < 0, phi + 2 * np.pi, phi)
    phi = np.where(phi >= 2 * np.pi, phi - 2 * np.pi, phi)
    ai = np.minimum((alpha / np.pi * size_alpha).astype(int), size_alpha - 1)
    pj = np.minimum((phi / 2 / np.pi * size_phi).astype(int), size_phi - 1)
    buckets = np.zeros((size_alpha, size_phi))
    np.add.at(buckets, (ai, pj), 1)

    a_c = (np.arange(size_alpha) + 0.5) / size_alpha * np.pi
    p_c = (np.arange(size_phi) + 0.5) / size_phi * 2 * np.pi
    A, P = np.meshgrid(a_c, p_c, indexing="ij")
    centres = np.stack([np.sin(A) * np.cos(P), np.sin(A) * np.sin(P), np.cos(A)], -1).reshape(-1, 3)
    val = np.asarray(value_fn(centres.astype(np.float32)), np.float64).reshape(size_alpha, size_phi)
    if sub <= 1:
        area = (2 * np.pi * np.sin(A) / size_phi) * (np.pi / size_alpha)
        theor = val * area * N / ddf_integral
    else:
        fa = (np.arange(size_alpha * sub) + 0.5) / (size_alpha * sub) * np.pi
        fp = (np.arange(size_phi * sub) + 0.5) / (size_phi * sub) * 2 * np.pi
        FA, FP = np.meshgrid(fa, fp, indexing="ij")
        pts = np.stack([np.sin(FA) * np.cos(FP), np.sin(FA) * np.sin(FP), np.cos(FA)], -1).reshape(-1, 3)
        fv = np.asarray(value_fn(pts.astype(np.float32)), np.float64).reshape(FA.shape)
        dA = np.sin(FA) * (np.pi / (size_alpha * sub)) * (2 * np.pi / (size_phi * sub))
        bucket_int = (fv * dA).reshape(size_alpha, sub, size_phi, sub).sum((1, 3))
        # the same quadrature's total replaces the Monte-Carlo integral, so the
        # expected counts are normalised consistently (a narrow light lobe
        # makes the 2e5-point MC estimate off by percents)
        ddf_integral = float(bucket_int.sum())
        theor = bucket_int * N / ddf_integral
    zero_nb = np.zeros_like(buckets, bool)
    for di, dj in ((1, 0), (-1, 0), (0, 1), (0, -1)):
        for i in range(size_alpha):
            ii = i + di
            if not 0 <= ii < size_alpha:
                continue
            jj = (np.arange(size_phi) + dj) % size_phi
            zero_nb[i] |= (buckets[ii, jj] == 0) | (val[ii, jj] == 0)
    use = (theor > 2) & (buckets >= 2) & ~zero_nb
    chi2 = float((((buckets - theor) ** 2) / np.where(use, theor, 1.0))[use].sum())
    dof = int(use.sum())
    lo, hi = 70 * dof / 100.0, 135 * dof / 100.0
    success = N / total_tries
    ok = (lo < chi2 < hi and 0.95 < success / ddf_integral < 1.05
          and (not strict_integral or 0.95 < ddf_integral < 1.05))
    return ok, dict(chi2=chi2, dof=dof, integral=ddf_integral, success=success)
