"""CPU oracle for the fancy_gym black-box reacher rollout path — TEST INFRASTRUCTURE ONLY.

Nothing in ``fancy_gym_crowd_amd`` imports, links or executes anything from this package:
it is the checker (tests/, ``__graft_entry__.smoke()``) and the CPU baseline leg of
``bench.py`` (``cpu_baseline``), never the thing measured or shipped.

Modules
-------
port      Structure-matched per-env restatement of the reference loop (numpy, same ops and
          dtypes as the reference, one Python object per env).  Pinned bit-exactly against
          the fixtures in tests/golden/ that were produced by the reference's own code
          (tests/golden/make_golden.py).  Also the ``cpu_baseline`` ("port").
fp32      Exact emulation of f32 fma chains / f32 rounding in numpy (matches MFMA f32
          numerics and the HIP VALU chains).
mp        Restatement of the movement-primitive math of mp_pytorch<=0.1.3 (ProMP / DMP /
          ProDMP, linear / exp phase, (zero-padded) normalized RBF, ProDMP precompute).
          mp_pytorch is NOT in the container and the reference's tests pin only structural
          properties: numeric MP parity to mp_pytorch is **parity unpinned** (SURVEY.md §8c).
batched   Vectorised (over envs) restatement of port + mp, used as the GPU parity oracle at
          thousands of envs; checked bit-exactly against ``port`` on small batches.
"""
