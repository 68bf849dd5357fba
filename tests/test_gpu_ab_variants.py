"""The A/B build (librt_amd_ab.so, `make ab`): every measured-and-rejected
scene-kernel variant still renders the oracle's images.

The shipped librt_amd.so carries only the default kernels; the A/B library is
loaded in ONE child process (a second copy of the ctypes binding cannot share
this process's), which runs tests/ab_variant_check.py over all variants.
"""
import json
import os
import subprocess
import sys

import pytest

import raytracingstudy_amd as rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(ROOT, "raytracingstudy_amd", "librt_amd_ab.so")


def test_shipped_library_refuses_ab_variants():
    # no GPU needed: rt_create validates the flags before touching a device
    with pytest.raises(rt._lib.RtError, match="variant not in this build"):
        rt.KernelRenderer(64, 48, mode="scene", spp=1, variant=rt._lib.VARIANT_PACKET)


@pytest.mark.gpu
def test_ab_variants_match_oracle(gpu):
    assert os.path.exists(AB_LIB), "build the A/B library first: make -C raytracingstudy_amd/csrc ab"
    env = dict(os.environ, RT_AMD_LIB=AB_LIB)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ab_variant_check.py")],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["ok"] and len(res["cases"]) == 36
