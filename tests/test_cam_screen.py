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
