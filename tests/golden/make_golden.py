"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Fixtures (inputs + expected outputs, all seeded):
  c1_known_answers.json  SURVEY.md 8c C4 hand-derived answers (written by hand,
                         not by this script; checked, never overwritten)
  c1_compat.npy          256x256 compat image, default pose, resize intrinsic
  compat_1080p.sha256    sha256 of the 1920x1080 compat image (default pose)
  scene_small.npz        96x64, 2 spp, 1k spheres (scene pose): rgba8,
                         radiance, counters; sha256 of the generated spheres/albedo
  scene_depth12.npz      80x60, 1 spp, 20k spheres, depth 12
The reference itself cannot be built or run here (DESIGN.md "Oracle"), so the
compat fixtures are pinned by c1_known_answers.json; the scene fixtures pin
the oracle's own spec against drift.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

SEED = 0x2545F491


def default_pose():
    p = np.zeros((4, 4), np.float32)
    p[0, 0], p[1, 1], p[2, 2], p[3, 3] = 1, -1, -1, 1
    p[3, :3] = (0, 0, 3)
    return p


def scene_pose():
    p = default_pose()
    p[3, :3] = (0.64, 0.64, 2.2)
    return p


def main():
    K = oracle.resize_intrinsic(256, 256)
    img = oracle.render_compat(256, 256, default_pose(), K)
    np.save(os.path.join(HERE, "c1_compat.npy"), img)
    K = oracle.resize_intrinsic(1920, 1080)
    big = oracle.render_compat(1920, 1080, default_pose(), K)
    with open(os.path.join(HERE, "compat_1080p.sha256"), "w") as f:
        f.write(hashlib.sha256(big.tobytes()).hexdigest() + "\n")

    for name, n, w, h, spp, depth in [("scene_small", 1000, 96, 64, 2, 7),
                                      ("scene_depth12", 20000, 80, 60, 1, 12)]:
        sp, al = oracle.generate_spheres(n, SEED)
        sc = oracle.Scene(sp, al, max_depth=depth)
        K = oracle.resize_intrinsic(w, h)
        rgba8, rad, cnt = sc.render(w, h, scene_pose(), K, spp=spp, seed=SEED)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rgba8=rgba8, radiance=rad,
                            counters=cnt,
                            spheres_sha256=np.frombuffer(hashlib.sha256(sp.tobytes()).digest(), np.uint8),
                            albedo_sha256=np.frombuffer(hashlib.sha256(al.tobytes()).digest(), np.uint8),
                            params=np.array([n, w, h, spp, depth, SEED], np.int64))
    print("goldens written to", HERE)


if __name__ == "__main__":
    main()
