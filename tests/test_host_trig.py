"""The observation fast path of k_episode_v2 (csrc/fgx_trig.h: fgx_sincos_fast, obs_trig_fast,
f32_checked) on the CPU: tests/host/obs_trig_check.hip compiles the same header for the host and, over
~1.75 M random samples (2, 5 and 8 links; angles up to 1e4, angles of 1e-9 and pi / 2 whose values sit
below the margin's f32 resolution), compares every f32 the fast path accepts with the exact path's
(libm cos / sin of the joint angles and of numpy's rounded cumulative angles, Env::fk's sequential
end-effector sums).  None may differ; |q| >= 2^20, inf and NaN must be refused; fgx_sincos_fast stays
within 2e-16 of long-double sin / cos.  (The device comparison against the exact kernels is
tests/test_gpu_info_rows.py.)"""
import json
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC), reason="no hipcc")
def test_obs_trig_fast_path_is_exact_when_it_accepts(tmp_path):
    exe = str(tmp_path / "obs_trig_check")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-Wno-unused-result",
                    os.path.join(HERE, "host", "obs_trig_check.hip"), "-o", exe], check=True)
    out = subprocess.run([exe, "1000000"], check=True, capture_output=True, text=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    assert r["checked_but_different"] == 0, r
    assert r["guard_failures"] == 0, r
    assert r["sincos_fast_max_abs_err"] < 2e-16, r
    samples = 1000000 + 500000 + 250000
    assert r["fallback_samples"] < 0.2 * samples, r   # (1/8 of the samples are built to fall back)
