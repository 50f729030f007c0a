"""CPU-baseline calibration: bench.py's cpu_baseline leg times oracle/port.py's
structure-matched per-env loop on the GPU box, because the reference cannot travel there.  This
script times, in ONE process on ONE core of this container, both:

  * "reference": the reference's own BlackBoxWrapper + SimpleReacherEnv(n_links=5) + PDController
    (black_box_wrapper.py:170-253, simple_reacher.py, pd_controller.py), imported from
    /root/reference through tests/golden/make_golden.py's gymnasium shim, with make_golden's
    StubTrajGen standing in for the absent mp_pytorch (table slices: no basis contraction);
  * "port": bench._cpu_worker, the loop bench.py runs on the GPU box (oracle/port.py, f32 ProMP
    contraction + forward difference per BB step);

alternating them in short slices so that clock / thermal drift hits both, and writes the ratio to
profiles/r06_cpu_calibration.json, which bench.py quotes in cpu_baseline.sample.

python tools/cpu_calibration.py [--seconds 12] [--slices 6] [--out profiles/r06_cpu_calibration.json]
"""
import argparse
import json
import os
import platform
import sys
import time

for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[k] = "1"

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def ref_runner(seed=0):
    """the shimmed reference's verbose-2 BB loop for fancy_ProMP/LongSimpleReacher-v0 shapes
    (envs/__init__.py:658-666: 5 links; PD gains 0.6 / 0.075 as registered for the ProMP variant)"""
    import make_golden as mg   # installs the shim, imports the reference modules
    raw = mg.make_raw("long")
    env = mg.SRMPWrapper(raw)
    rng = np.random.default_rng(seed)
    pos_t, vel_t = mg.smooth_tables(rng, 200, 5, 0.5, 1.0)
    tg = mg.StubTrajGen(25, pos_t, vel_t)
    bb = mg.BlackBoxWrapper(env, trajectory_generator=tg, tracking_controller=mg.PDController(0.6, 0.075),
                            duration=2.0)
    bb.reset(seed=seed)

    def run(seconds):
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            _, _, te, tr, info = bb.step(rng.standard_normal(25).astype(np.float32))
            tg.calls.clear()
            steps += int(info["trajectory_length"])
            if te or tr:
                bb.reset()
        return steps, time.perf_counter() - t0
    return run


def port_runner():
    import bench
    return lambda seconds: bench._cpu_worker((0, seconds))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=12.0, help="per leg, over all slices")
    ap.add_argument("--slices", type=int, default=6)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_cpu_calibration.json"))
    a = ap.parse_args()
    if hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    legs = {"reference": ref_runner(), "port": port_runner()}
    for run in legs.values():   # warm-up (imports, first allocations)
        run(0.5)
    tot = {k: [0, 0.0] for k in legs}
    per = a.seconds / a.slices
    for _ in range(a.slices):
        for k, run in legs.items():
            s, t = run(per)
            tot[k][0] += s
            tot[k][1] += t
    rate = {k: v[0] / v[1] for k, v in tot.items()}
    res = {
        "what": "inner env-steps/s on one core, same process, alternating slices: the shimmed reference's "
                "BlackBoxWrapper loop (stub trajectory generator, no MP contraction) vs bench.py's cpu_baseline "
                "worker (oracle/port.py with the f32 ProMP contraction)",
        "workload": "fancy_ProMP/LongSimpleReacher-v0 (5 links, T = 200, verbose 2, PD 0.6 / 0.075)",
        "reference_steps_per_s": rate["reference"],
        "port_steps_per_s": rate["port"],
        "port_over_reference": rate["port"] / rate["reference"],
        "seconds_per_leg": a.seconds, "slices": a.slices,
        "host": {"machine": platform.machine(), "processor": platform.processor(), "python": platform.python_version(),
                 "numpy": np.__version__, "cpu_count": os.cpu_count()},
        "note": "the reference leg's stub trajectory generator skips mp_pytorch's basis evaluation, so the "
                "reference rate is an upper bound of the real reference's; the port pays its contraction",
    }
    s = json.dumps(res, indent=1)
    print(s)
    with open(a.out, "w") as f:
        f.write(s + "\n")


if __name__ == "__main__":
    main()
