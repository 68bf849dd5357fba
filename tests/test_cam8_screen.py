"""The 8-byte image-plane screen of primary rays is sound (CPU; DESIGN.md 5.1
round 6 "An 8-byte image-plane screen for primary rays").

With RT_CAM8 a primary ray's chunk runs the exact ray-sphere tests only when
the lane's image-plane point s = (Bd).xy / (Bd).z lies within rho of the
sphere centre's projection q, both in the frame's basis B (rt_capi.cpp
cam8_basis), rho^2 stored as bf16 in the low bytes of the 8-byte record
{qx, qy} (cam8_screen_kernel).  rho bounds |q_a - q_b| <= sin(theta) /
(a_z cos(beta + theta)) for every direction within theta of the centre's,
plus the f32 errors of both points.  The oracle's test-only restatement
(orc_cam8_screen_check: the record as the kernel makes it, the lane's point
with each of the three f32 values next to 1/pz) counts exactly-accepted
pairs the screen rejects over rays aimed at sphere silhouettes from five
cameras: none at the product's rho, some with rho shrunk to 0.9, so the
check can see an unsound screen.
"""
import numpy as np
import pytest

import oracle
import raytracingstudy_amd as rt

from test_cam_screen import CAMERAS, _silhouette_rays


def _basis(o, target=(0.64, 0.64, 0.64)):
    """Rows x, y, z (z toward the target), orthonormal in f64, rounded to f32."""
    z = np.asarray(target, np.float64) - np.asarray(o, np.float64)
    if np.linalg.norm(z) < 1e-9:
        z = np.array([0.3, -0.2, 1.0])
    z /= np.linalg.norm(z)
    up = np.array([0.0, 1.0, 0.0]) if abs(z[1]) < 0.9 else np.array([1.0, 0.0, 0.0])
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.concatenate([x, y, z]).astype(np.float32)


@pytest.fixture(scope="module")
def spheres():
    sp, _ = rt.generate_spheres(100_000, rt.SEED)
    sp5, _ = rt.generate_spheres(1_000_000, rt.SEED)
    return np.concatenate([sp, sp5[:200_000]])


def _in_frame(B, d):
    """The frame contract cam8_basis checks: (Bd).z >= 0.1 |Bd|."""
    p = d.astype(np.float64) @ B.astype(np.float64).reshape(3, 3).T
    return p[:, 2] >= 0.1 * np.linalg.norm(p, axis=1)


@pytest.mark.parametrize("o", CAMERAS)
def test_image_plane_screen_never_rejects_an_accepted_sphere(spheres, o):
    B = _basis(o)
    rng = np.random.default_rng(abs(hash(("cam8",) + o)) % (1 << 32))
    miss = passed = exact = 0
    tight_miss = 0
    for spread in (1e-6, 1e-5, 1e-4, 1e-2, 0.5):
        d, idx = _silhouette_rays(o, spheres, 200_000, rng, spread)
        keep = _in_frame(B, d)
        d, idx = d[keep], idx[keep]
        m, p, e = oracle.cam8_screen_check(o, B, 1, d, spheres, idx)
        miss += m
        passed += p
        exact += e
        tight_miss += oracle.cam8_screen_check(o, B, 1, d, spheres, idx, shrink=0.9)[0]
    assert exact > 0 and passed >= exact
    assert miss == 0, f"screen rejected {miss} exactly-accepted pairs"
    # the negative control: rho 10% short of the bound rejects accepted pairs
    assert tight_miss > 0


def test_frame_outside_the_basis_passes_everything(spheres):
    """ok = 0 (cam8_basis found a ray behind or near B's image plane): every
    record is rho^2 = +inf, so every pair passes."""
    o = CAMERAS[0]
    rng = np.random.default_rng(11)
    d, idx = _silhouette_rays(o, spheres, 50_000, rng, 0.5)
    m, p, e = oracle.cam8_screen_check(o, _basis(o), 0, d, spheres, idx)
    assert m == 0 and p == d.shape[0]


def test_spheres_behind_or_around_the_camera_pass(spheres):
    """A camera inside a sphere, and spheres behind the image plane: their
    records pass every ray (the bound needs a_z > 0 and beta + theta < 1.45)."""
    s = spheres[7].astype(np.float64)
    o = tuple(np.float32(s[:3] + 0.3 * s[3]))
    B = _basis(o)
    rng = np.random.default_rng(5)
    d = rng.normal(size=(20_000, 3))
    d = (d / np.linalg.norm(d, axis=1)[:, None]).astype(np.float32)
    m, p, e = oracle.cam8_screen_check(o, B, 1, d, spheres, np.full(d.shape[0], 7, np.uint32))
    assert m == 0 and p == d.shape[0] and e == d.shape[0]
