"""Physics pins of the BxDF restatement (SURVEY §4 tier 6), one BSDF at a time.

The kernel oracle restates BSDFs.inc.hlsl (EvaluateBSDF / EvaluateBSDFPdf / SampleBSDF) and the
GPU reproduces it bit for bit, so what pins the oracle pins the GPU. These tests check the
restatement against properties the reference's BSDFs must have whatever the reading of the
HLSL -- closed forms, the agreement of the three functions with each other, the normalisation
of the sampling pdf, reciprocity, Fresnel at normal incidence -- in the frame n = (0,0,1),
t = (1,0,0) (oracle_bsdf_eval / oracle_bsdf_sample, test entries of the oracle). Tolerances
are statistical (stated per test) or a few float ulps where the property is exact.
"""
import numpy as np
import pytest

DIFFUSE, PLASTIC, CONDUCTOR, DIELECTRIC, THIN = 0, 1, 2, 3, 4


def _hemi(rng, n, lower=False):
    """Uniform directions on the upper (or lower) hemisphere."""
    z = rng.uniform(0.02, 1.0, n)
    phi = rng.uniform(0.0, 2.0 * np.pi, n)
    r = np.sqrt(1.0 - z * z)
    d = np.stack([r * np.cos(phi), r * np.sin(phi), -z if lower else z], 1)
    return d.astype(np.float32)


def _sphere(rng, n):
    z = rng.uniform(-1.0, 1.0, n)
    phi = rng.uniform(0.0, 2.0 * np.pi, n)
    r = np.sqrt(1.0 - z * z)
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], 1).astype(np.float32)


def _numbers(rng, n):
    return rng.uniform(0.0, 1.0, (n, 3)).astype(np.float32)


def test_lambert_closed_form(oracle_mod, golden_luts):
    """Diffuse: f = albedo / pi and pdf = cos(theta_i) / pi above the surface, 0 below; cosine
    sampling has E[cos theta] = 2/3, and every sample's f cos / pdf is the albedo."""
    rng = np.random.default_rng(1)
    a = (0.8, 0.5, 0.2)
    m = oracle_mod.bsdf_material(DIFFUSE, albedo=a)
    wi, wo = _hemi(rng, 4000), _hemi(rng, 4000)
    f, pdf = oracle_mod.bsdf_eval(golden_luts, m, wi, wo)
    np.testing.assert_allclose(f, np.broadcast_to(np.array(a, np.float32) / np.float32(np.pi), f.shape), rtol=2e-6)
    np.testing.assert_allclose(pdf, wi[:, 2] / np.pi, rtol=2e-6)
    f, pdf = oracle_mod.bsdf_eval(golden_luts, m, _hemi(rng, 1000, lower=True), _hemi(rng, 1000))
    assert not f.any() and not pdf.any()
    n = 200_000
    wi, f, pdf, delta = oracle_mod.bsdf_sample(golden_luts, m, _hemi(rng, n), _numbers(rng, n))
    assert not delta.any() and (pdf > 0).all() and (wi[:, 2] > 0).all()
    cos = wi[:, 2].astype(np.float64)
    assert abs(cos.mean() - 2.0 / 3.0) < 4.0 * cos.std() / np.sqrt(n)
    np.testing.assert_allclose(f * cos[:, None] / pdf[:, None], np.broadcast_to(a, f.shape), rtol=1e-5)


MATERIALS = [
    ("plastic_rough", dict(type=PLASTIC, albedo=(0.7, 0.6, 0.5), alpha=0.4, ior=1.5)),
    ("plastic_rough_ms", dict(type=PLASTIC, albedo=(0.7, 0.6, 0.5), alpha=0.6, ior=1.5, multiscattering=True)),
    ("conductor_rough", dict(type=CONDUCTOR, albedo=(3.9, 2.4, 1.6), alpha=0.35, ior=0.2)),
    ("conductor_rough_ms", dict(type=CONDUCTOR, albedo=(3.9, 2.4, 1.6), alpha=0.7, ior=0.2, multiscattering=True)),
    ("dielectric_rough", dict(type=DIELECTRIC, alpha=0.3, ior=1.5)),
    ("dielectric_rough_ms", dict(type=DIELECTRIC, alpha=0.5, ior=1.5, multiscattering=True)),
]


@pytest.mark.parametrize("name,kw", MATERIALS, ids=[m[0] for m in MATERIALS])
def test_sample_agrees_with_evaluate(oracle_mod, golden_luts, name, kw):
    """SampleBSDF's value and pdf are EvaluateBSDF's and EvaluateBSDFPdf's at the sampled
    direction (non-delta lobes): the three functions describe one BSDF."""
    rng = np.random.default_rng(2)
    m = oracle_mod.bsdf_material(**kw)
    n = 20_000
    wo = _hemi(rng, n)
    wi, f, pdf, delta = oracle_mod.bsdf_sample(golden_luts, m, wo, _numbers(rng, n))
    ok = ~delta & (pdf > 1e-4) & (np.abs(wi[:, 2]) > 1e-3)
    assert ok.mean() > 0.5
    fe, pe = oracle_mod.bsdf_eval(golden_luts, m, wi[ok], wo[ok])
    np.testing.assert_allclose(pe, pdf[ok], rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(fe, f[ok], rtol=2e-4, atol=1e-6)


@pytest.mark.parametrize("name,kw", MATERIALS, ids=[m[0] for m in MATERIALS])
def test_pdf_integrates_to_the_sampled_mass(oracle_mod, golden_luts, name, kw):
    """The pdf over the sphere of wi integrates to the probability that a sample is valid
    (the mass VNDF sampling loses below the surface, or to a zero value, is neither sampled
    nor counted): a uniform-sphere estimate of the integral against the sampler's own hit
    rate, within 5 standard errors."""
    rng = np.random.default_rng(3)
    m = oracle_mod.bsdf_material(**kw)
    for woz in (0.9, 0.5):
        wo1 = np.array([np.sqrt(1 - woz * woz), 0.0, woz], np.float32)
        n = 400_000
        wi = _sphere(rng, n)
        _, pdf = oracle_mod.bsdf_eval(golden_luts, m, wi, np.broadcast_to(wo1, wi.shape))
        est = pdf.astype(np.float64) * 4.0 * np.pi
        integral, se = est.mean(), est.std() / np.sqrt(n)
        k = 200_000
        wis, fs, ps, ds = oracle_mod.bsdf_sample(golden_luts, m, np.broadcast_to(wo1, (k, 3)), _numbers(rng, k))
        valid = (~ds & (ps > 0) & (fs.max(1) > 0)).mean()
        se2 = np.sqrt(valid * (1 - valid) / k)
        assert abs(integral - valid) < 5 * (se + se2) + 2e-3, (woz, integral, valid)
        assert integral < 1.0 + 5 * se


def test_conductor_is_reciprocal(oracle_mod, golden_luts):
    """A rough conductor's Cook-Torrance BRDF is symmetric in (wi, wo) (D, F(wo.h = wi.h) and
    G1(wi) G1(wo) over 4 cos cos), to float rounding."""
    rng = np.random.default_rng(4)
    m = oracle_mod.bsdf_material(CONDUCTOR, albedo=(3.9, 2.4, 1.6), alpha=0.3, ior=0.2)
    a, b = _hemi(rng, 5000), _hemi(rng, 5000)
    fab, _ = oracle_mod.bsdf_eval(golden_luts, m, a, b)
    fba, _ = oracle_mod.bsdf_eval(golden_luts, m, b, a)
    np.testing.assert_allclose(fab, fba, rtol=5e-5, atol=1e-7)


@pytest.mark.parametrize("ior", [1.33, 1.5, 2.4])
def test_smooth_dielectric_fresnel_at_normal_incidence(oracle_mod, golden_luts, ior):
    """A smooth dielectric seen head-on reflects with probability F0 = ((ior - 1) / (ior + 1))^2:
    the sampler's reflection rate, within 5 standard errors."""
    rng = np.random.default_rng(5)
    m = oracle_mod.bsdf_material(DIELECTRIC, alpha=0.0, ior=ior)
    n = 400_000
    wo = np.broadcast_to(np.array([0.0, 0.0, 1.0], np.float32), (n, 3))
    wi, f, pdf, delta = oracle_mod.bsdf_sample(golden_luts, m, wo, _numbers(rng, n))
    assert delta.all()
    refl = (wi[:, 2] > 0).mean()
    f0 = ((ior - 1) / (ior + 1)) ** 2
    assert abs(refl - f0) < 5 * np.sqrt(f0 * (1 - f0) / n), (refl, f0)


def test_white_furnace_bounds(oracle_mod, golden_luts):
    """Directional albedo E(wo) = E[f cos / pdf] of the reflecting BSDFs never exceeds 1 for a
    white, energy-conserving material (albedo 1 diffuse base under a dielectric coat; a
    conductor with eta -> 0 and k = 0, whose Fresnel term is 1), within 5 standard errors; at
    high roughness the single-scattering conductor loses energy (about 0.39 of it remains at
    alpha 0.9) and the Kulla-Conty term restores it to 1 within 0.01. (The test entry takes
    one eta: a conductor's other two channels have eta = 1, k = 0 and reflect nothing, so
    only channel x is checked for it.)"""
    rng = np.random.default_rng(6)
    n = 200_000
    wo = np.broadcast_to(np.array([0.6, 0.0, 0.8], np.float32), (n, 3))

    def albedo(**kw):
        m = oracle_mod.bsdf_material(**kw)
        wi, f, pdf, delta = oracle_mod.bsdf_sample(golden_luts, m, wo, _numbers(rng, n))
        w = np.where((pdf > 0)[:, None], f * np.abs(wi[:, 2:3]) / np.maximum(pdf, 1e-30)[:, None], 0.0).astype(np.float64)
        return w.mean(0), w.std(0) / np.sqrt(n)

    for kw in (dict(type=PLASTIC, albedo=(1, 1, 1), alpha=0.5, ior=1.5), dict(type=PLASTIC, albedo=(1, 1, 1), alpha=0.05, ior=1.5)):
        e, se = albedo(**kw)
        assert (e < 1.0 + 5 * se + 1e-3).all(), (kw, e)
    single, s1 = albedo(type=CONDUCTOR, albedo=(0.0, 0.0, 0.0), alpha=0.9, ior=1e-3)
    multi, s2 = albedo(type=CONDUCTOR, albedo=(0.0, 0.0, 0.0), alpha=0.9, ior=1e-3, multiscattering=True)
    single, s1, multi, s2 = single[0], s1[0], multi[0], s2[0]
    assert single < 0.9 and multi < 1.0 + 5 * s2 + 1e-3, (single, multi)
    assert abs(multi - 1.0) < 0.01 + 5 * s2, (single, multi)
