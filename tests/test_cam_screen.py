"""The camera-relative screen is sound (CPU; DESIGN.md 5.1 "Camera-relative
screen").

A primary ray's leaf chunk runs the exact ray-sphere tests only when the
screen fma(b, b, -C') >= 0 passes for some lane, with C' = |o - c|^2 - r^2
minus a slack of 16 u |o - c|^2 + 8 u r^2 (u = 2^-24), made per frame by
cam_screen_kernel.  The image is bit-exact only if the screen never rejects a
sphere the exact discriminant accepts.  The oracle's test-only restatement
of the screen (orc_cam_screen_check) counts such misses over rays aimed at
sphere silhouettes (where the two forms' rounding decides), from cameras
near, far, inside the box and inside spheres: none at the product's slack,
and some at zero slack, so the check can see an unsound screen.
"""
import numpy as np
import pytest

import oracle
import raytracingstudy_amd as rt

SLACK_OC, SLACK_R = 16.0, 8.0  # rt_params.h kScreenSlackOc / kScreenSlackR


def _unit_f32(w):
    """getRay's normalisation in f32: w / sqrtf(wx*wx + wy*wy + wz*wz)."""
    w = w.astype(np.float32)
    ww = (w[:, 0] * w[:, 0] + w[:, 1] * w[:, 1]) + w[:, 2] * w[:, 2]
    return (w / np.sqrt(ww)[:, None]).astype(np.float32)


def _silhouette_rays(o, sp, n, rng, spread):
    """n rays from o aimed at points c + p r (1 + xi) on random spheres'
    silhouettes (p a unit vector perpendicular to c - o), xi ~ U[-spread, spread]."""
    idx = rng.integers(0, sp.shape[0], n)
    c = sp[idx, :3].astype(np.float64)
    r = sp[idx, 3].astype(np.float64)
    v = c - np.asarray(o, np.float64)
    a = rng.normal(size=(n, 3))
    p = a - (np.sum(a * v, 1) / np.sum(v * v, 1))[:, None] * v
    p /= np.linalg.norm(p, axis=1)[:, None]
    xi = rng.uniform(-spread, spread, n)
    tgt = c + p * (r * (1.0 + xi))[:, None]
    return _unit_f32(tgt - np.asarray(o, np.float64)), idx


@pytest.fixture(scope="module")
def spheres():
    sp, _ = rt.generate_spheres(100_000, rt.SEED)
    sp5, _ = rt.generate_spheres(1_000_000, rt.SEED)
    return np.concatenate([sp, sp5[:200_000]])


CAMERAS = [
    (0.64, 0.64, 2.2),      # SURVEY 8d D2's scene camera
    (0.1, 1.2, -0.7),       # behind and to the side
    (0.64, 0.64, 0.64),     # inside the box
    (40.0, -25.0, 60.0),    # far
    (-3.0, 0.2, 0.5),
]


@pytest.mark.parametrize("o", CAMERAS)
def test_screen_never_rejects_an_accepted_sphere(spheres, o):
    rng = np.random.default_rng(abs(hash(o)) % (1 << 32))
    miss = passed = exact = 0
    for spread in (1e-6, 1e-5, 1e-4, 1e-2, 0.5):
        d, idx = _silhouette_rays(o, spheres, 200_000, rng, spread)
        m, p, e = oracle.cam_screen_check(o, d, spheres, idx, SLACK_OC, SLACK_R)
        miss += m
        passed += p
        exact += e
    assert miss == 0, f"screen rejected {miss} exactly-accepted pairs"
    assert exact > 0 and passed >= exact


def test_screen_inside_a_sphere_always_passes(spheres):
    """A camera inside a sphere: C' < 0, so every ray passes that sphere's screen."""
    s = spheres[7].astype(np.float64)
    o = tuple(np.float32(s[:3] + 0.3 * s[3]))
    rng = np.random.default_rng(5)
    d = _unit_f32(rng.normal(size=(10_000, 3)))
    idx = np.full(10_000, 7, np.uint32)
    miss, passed, exact = oracle.cam_screen_check(o, d, spheres, idx, SLACK_OC, SLACK_R)
    assert miss == 0 and passed == 10_000 and exact == 10_000


def test_check_sees_an_unsound_screen(spheres):
    """Without the slack, rounding makes the screen reject some silhouette
    pairs the exact discriminant accepts: the check above has teeth."""
    rng = np.random.default_rng(11)
    miss = 0
    for o in CAMERAS[:2]:
        d, idx = _silhouette_rays(o, spheres, 400_000, rng, 1e-6)
        miss += oracle.cam_screen_check(o, d, spheres, idx, 0.0, 0.0)[0]
    assert miss > 0


@pytest.mark.parametrize("which,bound", [("c3", 1.5), ("c5", 3.0)])
def test_slack_costs_a_thin_annulus(which, bound):
    """The slack widens each sphere's screen by an annulus: from the scene
    camera, over rays aimed uniformly at discs out to 1.5 radii, the screen
    passes 1.28x the pairs the exact test accepts for C3's spheres (r ~
    0.003) and 1.83x for C5's 1M spheres (r ~ 0.0015; the slack is relative
    to |o - c|^2, so small spheres pay more)."""
    n = 100_000 if which == "c3" else 1_000_000
    sp, _ = rt.generate_spheres(n, rt.SEED)
    rng = np.random.default_rng(3)
    d, idx = _silhouette_rays(CAMERAS[0], sp, 400_000, rng, 0.5)
    miss, passed, exact = oracle.cam_screen_check(CAMERAS[0], d, sp, idx, SLACK_OC, SLACK_R)
    assert miss == 0 and exact <= passed <= bound * exact, (passed / exact)


# ---- light-plane shadow screen (DESIGN.md 5.1 "Light-plane screen") --------

SLACK_M, GROW = 64.0, 4.0  # rt_params.h kShadowSlackM; shd_screen_kernel's r (1 + 4u) and (1 + 4u)


def _kernel_light(ld):
    """FrameArgs::L as rt_capi.cpp fill_frame_args makes it: -(ld / |ld|) in f32."""
    ld = np.asarray(ld, np.float32)
    ll = np.sqrt((ld[0] * ld[0] + ld[1] * ld[1]) + ld[2] * ld[2])
    return (-(ld / ll)).astype(np.float32)


def _shadow_pairs(sp, L, n, rng, spread, big_m):
    """n shadow-ray origins whose rays (direction L) pass sphere idx[k] at
    r (1 + xi) from its centre, xi ~ U[-spread, spread], the origin anywhere
    along the line within the scene's bound M (in front of or behind it)."""
    l = L.astype(np.float64) / np.linalg.norm(L.astype(np.float64))
    a = np.array([1.0, 0.0, 0.0]) if abs(l[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
    e1 = a - (a @ l) * l
    e1 /= np.linalg.norm(e1)
    e2 = np.cross(l, e1)
    idx = rng.integers(0, sp.shape[0], n)
    c = sp[idx, :3].astype(np.float64)
    r = sp[idx, 3].astype(np.float64)
    th = rng.uniform(0, 2 * np.pi, n)
    xi = rng.uniform(-spread, spread, n)
    w = (np.cos(th)[:, None] * e1 + np.sin(th)[:, None] * e2) * (r * (1.0 + xi))[:, None]
    s = rng.uniform(-1.0, 1.0, n)
    o = (c + w + s[:, None] * l).astype(np.float32)
    keep = np.linalg.norm(o.astype(np.float64), axis=1) <= big_m
    return o[keep], idx[keep]


def _bound(sp):
    lo = (sp[:, :3] - sp[:, 3:]).min(0).astype(np.float64)
    hi = (sp[:, :3] + sp[:, 3:]).max(0).astype(np.float64)
    return max(np.linalg.norm(np.where([(c >> i) & 1 for i in range(3)], hi, lo)) for c in range(8))


LIGHTS = [(1.0, 1.0, -1.0),      # the default
          (0.3, -2.0, 0.7), (0.0, 0.0, 1.0), (-1.0, 1e-3, 0.2)]


@pytest.mark.parametrize("ld", LIGHTS)
def test_shadow_screen_never_rejects_an_accepted_sphere(spheres, ld):
    """The light-plane screen at the product's slack passes every sphere whose
    exact discriminant (isect, direction L) accepts it, for shadow rays passing
    sphere silhouettes; at zero slack it misses some (the check has teeth)."""
    L = _kernel_light(ld)
    big_m = _bound(spheres)
    rng = np.random.default_rng(11)
    miss = passed = exact = miss0 = 0
    for spread in (1e-7, 1e-6, 1e-5, 1e-3, 0.3):
        o, idx = _shadow_pairs(spheres, L, 200_000, rng, spread, big_m)
        m, p, e = oracle.shd_screen_check(o, L, spheres, idx, big_m, SLACK_M, GROW)
        miss += m
        passed += p
        exact += e
        miss0 += oracle.shd_screen_check(o, L, spheres, idx, big_m, 0.0, 0.0)[0]
    assert miss == 0, f"shadow screen rejected {miss} exactly-accepted pairs"
    assert exact > 0 and passed >= exact
    if np.count_nonzero(ld) > 1:  # an axis-aligned L makes both forms exact
        assert miss0 > 0, "zero slack should miss some silhouette pairs"


def test_shadow_screen_annulus():
    """What the slack costs: shadow rays spread uniformly over discs of 1.5
    radii around C3's and C5's spheres pass the screen at most a few percent
    more often than the exact test accepts them."""
    L = _kernel_light((1.0, 1.0, -1.0))
    rng = np.random.default_rng(3)
    for n_sph in (100_000, 1_000_000):
        sp, _ = rt.generate_spheres(n_sph, rt.SEED)
        big_m = _bound(sp)
        o, idx = _shadow_pairs(sp, L, 400_000, rng, 0.0, big_m)
        # redraw each pair's offset uniformly over the disc of radius 1.5 r
        l = L.astype(np.float64) / np.linalg.norm(L.astype(np.float64))
        c = sp[idx, :3].astype(np.float64)
        t = (o.astype(np.float64) - c) @ l
        w = o.astype(np.float64) - c - t[:, None] * l
        w /= np.linalg.norm(w, axis=1)[:, None]
        rad = sp[idx, 3].astype(np.float64) * np.sqrt(rng.uniform(0, 2.25, len(idx)))
        o2 = (c + w * rad[:, None] + t[:, None] * l).astype(np.float32)
        m, p, e = oracle.shd_screen_check(o2, L, sp, idx, big_m, SLACK_M, GROW)
        assert m == 0
        print(n_sph, "passed / accepted", p / e)
        assert p <= 1.05 * e, (n_sph, p, e)


@pytest.mark.parametrize("ld", LIGHTS)
def test_packed_shadow_screen_never_rejects_an_accepted_sphere(spheres, ld):
    """The same with each sphere's own rr' packed as bf16 into the low bytes of
    its 8-byte {u, v} record (RT_SHD8_PER, oracle.c orc_shd8_screen_check):
    no miss at the product's radius, some with it shrunk by 1%."""
    L = _kernel_light(ld)
    big_m = _bound(spheres)
    rng = np.random.default_rng(13)
    miss = passed = exact = tight = 0
    for spread in (1e-7, 1e-6, 1e-5, 1e-3, 0.3):
        o, idx = _shadow_pairs(spheres, L, 200_000, rng, spread, big_m)
        m, p, e = oracle.shd8_screen_check(o, L, spheres, idx, big_m, SLACK_M, GROW)
        miss += m
        passed += p
        exact += e
        tight += oracle.shd8_screen_check(o, L, spheres, idx, big_m, SLACK_M, GROW, shrink=0.9)[0]
    assert miss == 0, f"packed shadow screen rejected {miss} exactly-accepted pairs"
    assert exact > 0 and passed >= exact
    assert tight > 0
