"""Benchmark: inner env-steps/s of fancy_ProMP/LongSimpleReacher-v0 black-box steps on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--global-envs G | --envs ENVS_PER_GPU]

BASELINE.json's metric is quoted at N = 65536 envs in total over 1/2/4/8 GPUs: the default is
STRONG scaling (--global-envs 65536, each of the N ranks owns 65536/N envs).  --envs gives every
rank a fixed number of envs instead (weak scaling).  With N > 1 the strong-scaling line also
carries a weak-scaling measurement (65536 envs per GPU) as a secondary field.
For N > 1, `bench.py --gpus N` starts the N ranks itself (torch.distributed.run as a child process,
one process per GPU) unless a launcher already did (WORLD_SIZE set; it must equal --gpus); with
fewer visible GPUs than ranks they share cuda:0 over gloo (rehearsal).  Env shards are independent
(seeds = global env index, the rank's rows of the global parameter matrix); the only exchange is an
RCCL all_gather of the episode returns after EVERY BB step (one episode each), captured with the
episode launches in one HIP graph and inside the timed window.  Prints ONE JSON line on rank 0.

A "step" = one BlackBoxWrapper.step for every env (black_box_wrapper.py:170-253): MP trajectory
(200 samples), PD control, 200 reacher substeps, return, VectorEnv auto-reset.
The metric counts inner env steps = sum of trajectory_length over envs and steps.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "inner env-steps/sec, ProMP 5-link Reacher, N=65536 envs at 1/2/4/8 MI355X"
WORKLOAD = "fancy_ProMP/LongSimpleReacher-v0"
GLOBAL_ENVS = 65536
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_VEC_PEAK_TF = 157.3   # MI355X_MICROARCH.md: Peak FP32 (vector / matrix f32)
CLOCK_GHZ = 2.4            # MI355X peak engine clock (GRBM_GUI_ACTIVE / kernel time agrees, profiles/)
# VALU issue, architectural (MI355X_MICROARCH.md, Execution model + per-instruction constants): a
# wave64 VALU instruction occupies its SIMD-32 for 2 cycles (f32 / int / packed f32); an f64 op or a
# conversion runs at the 78.6 TF f64 vector rate, 4 cycles.  The peak of a kernel is 1 / (its
# PMC-weighted mean of these costs).  tools/valu_rates.hip measures what the hardware sustains
# beside it: 4.68 cycles per f64 instruction with >= 4 independent waves per SIMD, 6.12 for a lone
# wave (profiles/r01_valu_rates.jsonl) -- reported as secondary fields, never as the peak.
ISSUE_F64_CYCLES = 4.0
ISSUE_F32_CYCLES = 2.0
ISSUE_SIMD_CYCLES = 4.68
ISSUE_SINGLE_WAVE_CYCLES = 6.12
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")


def lib_build_id():
    from fancy_gym_crowd_amd import _lib
    return _lib.load().fgx_build_id().decode()


def pmc_entry(env_id, n_envs, kernel, build_id):
    """Committed rocprofv3 PMC summary (tools/pmc_summary.py) of the kernel this run launches, for
    the library build that runs: VALU instructions (and their f64 / conversion mix) and HBM bytes
    per launch.  Returns (entry or None, note)."""
    try:
        with open(PMC_SUMMARY) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None, "no profiles/pmc_summary.json"
    stale = None
    for e in entries:
        if e.get("workload") == env_id and int(e.get("envs", -1)) == n_envs and e.get("kernel") == kernel:
            if e.get("build_id") == build_id:
                return e, "pmc of this build"
            stale = e.get("build_id")
    if stale is not None:
        return None, f"pmc entry is of build {stale}, the library is {build_id}: rejected"
    return None, "no committed PMC pass for this kernel and size"


def valu_issue_peak(pmc):
    """Architectural VALU issue peak (wave-instructions / cycle / SIMD) for the kernel's measured
    instruction mix: f64 + conversions at 4 cycles, everything else at 2."""
    mix = pmc.get("valu_mix")
    total = float(pmc["valu_instr_per_launch"])
    if mix:
        slow = float(mix["f64"]) + float(mix["cvt"])
        source = pmc.get("valu_mix_source", "PMC")
    else:   # DESIGN.md section 5 mix of k_episode: 58 f64 + 10 cvt of 114 per inner step
        slow = total * 68.0 / 114.0
        source = "DESIGN.md static mix (no PMC mix counters in the entry)"
    slow = min(slow, total)
    cyc = (ISSUE_F64_CYCLES * slow + ISSUE_F32_CYCLES * (total - slow)) / total
    return 1.0 / cyc, cyc, slow / total, source


def episode_bytes_per_env(env):
    """Algorithmic HBM bytes of one episode launch per env (info_level 0, autoreset on)."""
    n, P, out = env.dof, env.n_params, env.out_dim
    hole = 0 if env._eng.cfg.env_kind == 0 else 3 * 8      # SimpleReacher kernels skip hole / aux
    state = 2 * n * 8 + 2 * 8 + hole + 3 * 4 + 5 * 8       # q, qd, goal, [hole], steps/plans/flags, rng
    reads = P * 4 + state
    writes = state + 8 + 2 * out * 4 + 8 + 1 + 1 + 4       # state + start angle, obs, final_obs, ret, flags, len
    return reads + writes


def env_id_of(env):
    return env.meta["env_id"]


def basis_gemm_fields(N, T, n, nb, n_params, t, pmc):
    """The basis GEMM's accounting from its launch time t (s) and its committed PMC entry (or None).
    Algorithmic work: ONE contraction per env, plan = table [T, nb] x weights [nb, dof] (ProMP: the
    velocities are a forward difference of the positions, no second GEMM), 2 nb T dof flops per env.
    What the matrix cores issue is the MFMA-padded count (K = 8 for nb = 5, 8 tiles of 28 rows for
    T = 200): SQ_INSTS_VALU_MFMA_MOPS_F32 of the PMC pass.  mfma_frac = those issued flops over the
    launch time, against the f32 matrix peak."""
    flops = 2 * nb * T * n * N
    out_bytes = 2 * 4 * N * T * n + 4 * N * n_params
    out = {"flops_algorithmic": flops, "us": t * 1e6, "algorithmic_tflops": flops / t / 1e12,
           "peak_tflops": FP32_VEC_PEAK_TF, "hbm_GBps": out_bytes / t / 1e9,
           "hbm_frac": out_bytes / t / 1e9 / HBM_PEAK_GBS, "pmc": None}
    if pmc is not None and pmc.get("mfma_f32_flops"):
        issued = float(pmc["mfma_f32_flops"])
        out["pmc"] = {"mfma_f32_instr": pmc.get("mfma_f32_instr"), "mfma_f32_flops_issued": issued,
                      "mfma_busy_cycles": pmc.get("mfma_busy_cycles"),
                      "issued_over_algorithmic": issued / flops,
                      "traffic_bytes_per_launch": pmc.get("traffic_bytes_per_launch"),
                      "kernel_ns_under_pmc": (pmc.get("kernel_ns_median_under_pmc") or {}).get("mfma"),
                      "source": pmc.get("source")}
        out["mfma_tflops"] = issued / t / 1e12
        out["mfma_frac"] = issued / t / 1e12 / FP32_VEC_PEAK_TF
        out["mfma_frac_source"] = "PMC-issued MFMA flops of this build / launch time"
    else:   # no PMC pass of this build: the algorithmic count (a lower bound of what is issued)
        out["mfma_tflops"] = flops / t / 1e12
        out["mfma_frac"] = flops / t / 1e12 / FP32_VEC_PEAK_TF
        out["mfma_frac_source"] = "algorithmic flops / launch time (no PMC pass of this build)"
    return out


def basis_gemm(env, params, reps=10):
    """The MP basis x weights contraction as its own launch (BlackBoxWrapper.get_trajectory ->
    fgx_trajectory -> k_traj_mfma, v_mfma_f32_32x32x2_f32 with K = 8): time per launch from HIP
    events around a graph replay of `reps` launches, MFMA utilisation against the f32 matrix peak
    (basis_gemm_fields) and the HBM rate of its [N, T, dof] f32 outputs."""
    import ctypes

    import torch
    N, T, n = env.num_envs, env.T, env.dof
    pos = torch.empty((N, T, n), dtype=torch.float32, device=params.device)
    vel = torch.empty_like(pos)
    lib, h = env._eng.lib, env._eng.h
    args = [ctypes.c_void_p(x.data_ptr()) for x in (params, pos, vel)]
    launch = lambda: lib.fgx_trajectory(h, *args, env._eng.stream())   # noqa: E731
    launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    pmc, note = pmc_entry(env_id_of(env), N, "k_traj_mfma", lib_build_id())
    out = {"kernel": "k_traj_mfma", "pmc_note": note}
    out.update(basis_gemm_fields(N, T, n, env._eng.cfg.n_basis, env.n_params, t, pmc))
    out["note"] = ("K = 8 (5 basis + zero pad): arithmetic intensity 2 flop/B, bound by the output write; the fused "
                   "episode kernels evaluate the same contraction in registers instead")
    return out


# ----------------------------------------------------------------------------- CPU baseline
def cpu_share():
    """CPUs this job may use: the affinity mask, capped by a cgroup CPU quota (cgroup v2
    cpu.max / v1 cfs_quota) when one is set.  Returns (cpus, affinity, source)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None and quota < aff:
        return max(1, int(quota)), aff, f"cgroup CPU quota {quota:g} (affinity {aff})"
    return aff, aff, f"sched_getaffinity ({aff})"


def cpu_baseline(seconds=12.0, cores=None):
    """The oracle port (structure-matched per-env Python loop of the reference) on host cores:
    one process per usable CPU (cpu_share), each running the loop for `seconds`."""
    import multiprocessing as mp_
    n, aff, source = cpu_share()
    cores = cores or n
    ctx = mp_.get_context("fork")   # called before this process touches the GPU (main())
    with ctx.Pool(cores) as pool:
        t0 = time.perf_counter()
        res = pool.map(_cpu_worker, [(i, seconds) for i in range(cores)])
        wall = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    per_core = float(np.mean([r[0] / r[1] for r in res]))
    calib, cal_note = None, "no committed calibration"
    try:   # tools/cpu_calibration.py: this worker vs the shimmed reference, one core, one process
        with open(os.path.join(ROOT, "profiles", "r06_cpu_calibration.json")) as f:
            cj = json.load(f)
        calib = {k: cj[k] for k in ("reference_steps_per_s", "port_steps_per_s", "port_over_reference")}
        calib["source"] = "profiles/r06_cpu_calibration.json (tools/cpu_calibration.py, build container)"
        cal_note = (f"calibrated in the build container against the shimmed reference (stub MP): this worker runs "
                    f"{cj['port_over_reference']:.3f}x the reference loop's rate on the same core")
    except (OSError, ValueError, KeyError):
        pass
    return dict(value=steps / wall, unit="inner env-steps/s", cores=cores, kind="port",
                per_core=per_core, affinity_cpus=aff, cores_source=source, calibration=calib,
                sample=f"oracle/port.py per-env loop (f32 ProMP contraction + PD + 200 substeps with the "
                       f"reference's per-step numpy ops incl. its 2 self-collision checks + autoreset), "
                       f"{WORKLOAD}, {cores} processes x ~{seconds:.0f}s, {steps} inner steps; "
                       f"os.cpu_count()={os.cpu_count()}, usable CPUs from {source}; {cal_note}")


def _cpu_worker(args):
    wid, seconds = args
    from oracle import mp, port
    spec = mp.MPSpec("promp", 5, 5, "linear", 2.0, zero_start=1)
    tables = mp.build_tables(spec, 202)
    rng = np.random.default_rng(1234 + wid)

    phi = tables["phi"][1:201]                       # [T, nb] f32
    dt32 = tables["dt32"][1:200, None]

    def traj(params, t0, q, qd):
        # mp_pytorch-cost ProMP evaluation (one f32 contraction + forward difference per BB step);
        # the bit-exact fma-chain emulation of oracle/mp.py is a checker, not a cost model
        w = params.reshape(5, 5)
        pos = (phi @ w.T).astype(np.float32)
        vel = np.empty_like(pos)
        vel[:-1] = (pos[1:] - pos[:-1]) / dt32
        vel[-1] = vel[-2]
        return pos, vel
    env = port.Reacher("LongSimpleReacher")
    bb = port.BlackBoxPort(env, traj, port.PD(0.6, 0.075), verbose=2)
    bb.reset(seed=wid)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, _, te, tr, info = bb.step(rng.standard_normal(spec.n_params, dtype=np.float32))
        steps += info["trajectory_length"]
        if te or tr:
            bb.reset()
    return steps, time.perf_counter() - t0


# ----------------------------------------------------------------------------- GPU run
def run_shard(env_id, n_local, rank, world, K, W, use_graph, dev, dist, coll_dev, overlap="auto"):
    """K timed BB steps of this rank's shard (global envs [rank * n_local, (rank + 1) * n_local)),
    bracketed by barrier + synchronize on both sides.  Returns wall time (max over ranks), inner
    steps (sum over ranks), this rank's event time per step, inner steps and the env."""
    import torch

    import fancy_gym_crowd_amd as fgx
    from fancy_gym_crowd_amd import shard
    N = n_local
    lo, _ = shard.shard_range(N, rank, world)
    env = fgx.make(env_id, num_envs=N, device=dev, seed_offset=lo, info_level=0)
    P = env.n_params
    # MP parameters: default_rng(1234).standard_normal((N_global, P), f32), this rank's rows
    allp = np.random.default_rng(1234).standard_normal((N * world, P), dtype=np.float32)
    params = torch.from_numpy(shard.shard_rows(allp, rank, world).copy()).to(dev)
    env.reset(seed=0)
    obs = torch.empty((N, env.out_dim), dtype=torch.float32, device=dev)
    fobs = torch.empty_like(obs)
    ret = torch.empty(N, dtype=torch.float64, device=dev)
    te = torch.empty(N, dtype=torch.uint8, device=dev)
    tr = torch.empty(N, dtype=torch.uint8, device=dev)
    tl = torch.empty(N, dtype=torch.int32, device=dev)
    acc = env.new_inner_steps()   # device counter of inner env steps
    # every BB step ends with the episode-return all_gather over RCCL/xGMI (the path's only
    # exchange): one all_gather_into_tensor of this rank's [N] f64 returns.  Two
    # schedules of the same work: "inline" (the gather follows its episode kernel on the launch
    # stream) and "overlap" (returns double-buffered, gather k on a side stream while episode
    # k + 1 runs; step k + 2 waits for gather k before it overwrites that buffer).  With
    # --overlap auto both are captured, each replayed once untimed, and the one whose slowest
    # rank is faster is timed (the same choice on every rank).  The gloo rehearsal (host buffers)
    # gathers in line, eagerly.
    gbuf = torch.empty(N * world, dtype=torch.float64, device=coll_dev) if dist is not None else None
    can_overlap = gbuf is not None and gbuf.is_cuda and overlap != "off"
    rets = [ret, torch.empty_like(ret)] if can_overlap else [ret, ret]
    gbufs = [gbuf, torch.empty_like(gbuf)] if can_overlap else [gbuf, gbuf]
    comm = torch.cuda.Stream(device=dev) if can_overlap else None
    st = {"k": 0, "gathers": 0, "free": [None, None], "pending": False}

    def bb_step(ov, count=True):
        s = st["k"] % 2 if ov else 0
        st["k"] += 1
        if ov and st["free"][s] is not None:
            torch.cuda.current_stream().wait_event(st["free"][s])
        env.step_into(params, obs, rets[s], te, tr, tl, fobs, inner_steps=acc if count else None)
        if gbuf is None:
            return
        st["gathers"] += 1
        if not ov:
            shard.gather_returns_into(gbufs[s], rets[s])
            return
        ready = torch.cuda.Event()
        ready.record()
        comm.wait_event(ready)
        with torch.cuda.stream(comm):
            shard.gather_returns_into(gbufs[s], rets[s])
            done = torch.cuda.Event()
            done.record()
        st["free"][s] = done
        st["pending"] = True

    def join():
        """the launch stream waits for the gathers still in flight on the side stream"""
        if st["pending"]:
            torch.cuda.current_stream().wait_stream(comm)
        st["free"], st["pending"] = [None, None], False

    for _ in range(W):
        bb_step(False, count=False)
    torch.cuda.synchronize()
    st["gathers"] = 0

    def capture(fn):
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(K):
                    fn()
                join()
            torch.cuda.synchronize()
            return g, None
        except Exception as e:   # capture unsupported: eager launches instead
            torch.cuda.synchronize()
            return None, str(e)

    def timed_graph(g, fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if g is not None:
            g.replay()
        else:
            for _ in range(K):
                fn()
            join()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K

    # the return gather alone (K captured all_gathers): the collective's own cost per BB step
    gather_ms = None
    if gbuf is not None and gbuf.is_cuda and use_graph:
        cg, _ = capture(lambda: shard.gather_returns_into(gbuf, ret))
        if cg is not None:
            gather_ms = timed_graph(cg, None)
            del cg

    # kernel-only time: the K episode launches alone in a HIP graph, HIP events on the launch stream
    # (outside the timed region; it separates kernel time from the per-step collective)
    kstep = lambda: env.step_into(params, obs, ret, te, tr, tl, fobs)   # noqa: E731
    kgraph = capture(kstep)[0] if use_graph else None
    kern_ms = timed_graph(kgraph, kstep)
    del kgraph

    # the timed BB steps: K x (episode launch [+ return all_gather]).  RCCL collectives on device
    # buffers are captured into the same HIP graph as the kernels; the gloo rehearsal (host
    # buffers) cannot be captured and runs eagerly.
    graph, gerr, ov = None, None, overlap == "on" and can_overlap
    trial = {}
    if use_graph and (gbuf is None or gbuf.is_cuda):
        modes = [False, True] if (overlap == "auto" and can_overlap) else [ov]
        graphs = {}
        for m in modes:
            st["gathers"] = 0
            g, e = capture(lambda: bb_step(m))
            if g is None:
                gerr = e
                continue
            graphs[m] = (g, st["gathers"])
        if len(graphs) == 2:   # one untimed replay of each, slowest rank decides, same pick everywhere
            t_in = timed_graph(graphs[False][0], None)
            t_ov = timed_graph(graphs[True][0], None)
            if dist is not None:
                t_in, t_ov = [max(x) for x in zip(*shard.gather_floats([t_in, t_ov], coll_dev))]
            trial = {"inline_ms_per_step": t_in, "overlap_ms_per_step": t_ov}
            ov = t_ov < t_in
        elif graphs:
            ov = next(iter(graphs))
        if graphs:
            graph, n_captured = graphs[ov]
            graphs.clear()
        elif gerr:
            print(f"[bench] graph capture failed ({gerr}); timing eager launches", file=sys.stderr)
    if graph is None:
        n_captured = 0
    st["gathers"] = 0
    acc.zero_()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
        st["gathers"] = n_captured
    else:
        for _ in range(K):
            bb_step(ov)
        join()
    ev1.record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0          # closing barrier below is outside this window
    step_ms = ev0.elapsed_time(ev1) / K
    barrier_ms = 0.0
    if dist is not None:
        tb = time.perf_counter()
        dist.barrier()
        barrier_ms = (time.perf_counter() - tb) * 1e3
    inner_local = int(acc.sum().item())
    coll_ms = max(0.0, step_ms - kern_ms) if dist is not None else 0.0
    timing_local = [kern_ms, step_ms, coll_ms, barrier_ms, elapsed * 1e3, float(st["gathers"]),
                    -1.0 if gather_ms is None else gather_ms]
    if dist is not None:
        elapsed = shard.max_over_ranks(elapsed, coll_dev)
        inner = shard.sum_over_ranks(inner_local, coll_dev)
        shards = shard.gather_ints([lo, lo + N, inner_local], coll_dev)
        timing = shard.gather_floats(timing_local, coll_dev)
    else:
        inner = inner_local
        shards = [[lo, lo + N, inner_local]]
        timing = [timing_local]
    per_rank = [{"rank": i, "kernel_ms_per_step": t[0], "step_ms": t[1], "exposed_collective_ms_per_step": t[2],
                 "gather_ms": None if t[6] < 0 else t[6], "barrier_ms": t[3], "wall_ms": t[4], "gathers": int(t[5])}
                for i, t in enumerate(timing)]
    launch = "hip graph of the K steps" if graph is not None else "eager"
    if gbuf is not None:
        launch += " (episode kernel + return all_gather per BB step"
        launch += (", gather k overlapped with episode k + 1 on a side stream" if ov else ", in line")
        launch += (", captured)" if graph is not None else ")")
    return dict(elapsed=elapsed, inner=inner, inner_local=inner_local, kern_ms=kern_ms, env=env, params=params,
                shards=shards, per_rank=per_rank, launch=launch, gathers=st["gathers"], capture_error=gerr,
                schedule_trial=trial)


def roofline(env_id, env, N, kern_ms, inner_local, K, simds, build_id):
    """Roofline of the episode kernel.  Its state stays in registers for all T substeps, so the
    binding resource is VALU instruction issue: achieved = VALU wave-instructions per SIMD per
    clock over the kernel time (instruction count from the committed rocprofv3 PMC pass of this
    kernel, size and library build), peak = the architectural issue rate for the kernel's PMC
    instruction mix (valu_issue_peak).  HBM is reported beside it."""
    kernel = env.episode_kernel()
    bpe = episode_bytes_per_env(env)
    hbm_gbs = bpe * N / (kern_ms * 1e-3) / 1e9
    pmc, pmc_note = pmc_entry(env_id, N, kernel, build_id)
    hbm = {"achieved_GBps": hbm_gbs, "peak_GBps": HBM_PEAK_GBS, "frac": hbm_gbs / HBM_PEAK_GBS,
           "algorithmic_bytes_per_env": bpe, "algorithmic_bytes_per_launch": bpe * N,
           "bytes_per_inner_step": bpe * N / max(1, inner_local / K)}
    out = {"kernel": kernel, "kernel_ms": kern_ms, "build_id": build_id, "pmc_note": pmc_note, "hbm": hbm}
    if pmc is not None:
        cyc = kern_ms * 1e-3 * CLOCK_GHZ * 1e9
        achieved = pmc["valu_instr_per_launch"] / simds / cyc
        peak, peak_cyc, slow_frac, mix_source = valu_issue_peak(pmc)
        traffic = pmc.get("traffic_bytes_per_launch")
        hbm["traffic_over_algorithmic"] = traffic / (bpe * N) if traffic else None
        out.update({"bound": "valu_issue", "achieved": achieved, "peak": peak,
                    "unit": "VALU wave-instr/cycle/SIMD", "frac": achieved / peak, "traffic": traffic,
                    "peak_note": f"peak = 1/{peak_cyc:.3f}: f64 + cvt ({slow_frac:.3f} of the VALU instructions, "
                                 f"{mix_source}) at {ISSUE_F64_CYCLES:g} cycles, the rest at {ISSUE_F32_CYCLES:g} "
                                 f"(MI355X_MICROARCH.md); clock {CLOCK_GHZ} GHz",
                    "secondary": {"frac_vs_measured_4wave_floor": achieved * ISSUE_SIMD_CYCLES,
                                  "frac_vs_lone_wave_floor": achieved * ISSUE_SINGLE_WAVE_CYCLES,
                                  "floors_source": "tools/valu_rates.hip, profiles/r01_valu_rates.jsonl"},
                    "pmc": {k: pmc.get(k) for k in ("valu_instr_per_launch", "valu_instr_per_inner_step_per_env",
                                                    "valu_mix", "valu_busy_pct", "waves",
                                                    "kernel_ns_median_under_pmc", "build_id", "source")}})
    else:   # no PMC pass of this kernel / size / build committed: the HBM roofline alone
        out.update({"bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm_gbs / HBM_PEAK_GBS, "traffic": None})
    return out


def spawn_ranks(n, argv):
    """`bench.py --gpus N` outside a torch.distributed launcher: start the N ranks (one process
    per GPU) with torch.distributed.run as a child of this process -- which has not touched the GPU
    -- and return their exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["FGX_BENCH_SPAWNED"] = "1"
    print(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a torch.distributed launcher bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-envs", type=int, default=GLOBAL_ENVS,
                    help="total envs over all ranks (strong scaling, the metric's definition)")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (weak scaling instead)")
    ap.add_argument("--env-id", default=WORKLOAD)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-weak", action="store_true", help="skip the secondary weak-scaling measurement")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="launch the K steps eagerly instead of replaying them as one HIP graph")
    ap.add_argument("--overlap", choices=("auto", "on", "off"), default="auto",
                    help="N > 1 (RCCL): run each BB step's return all_gather in line after its episode kernel "
                         "(off), overlapped with the next step's kernel on a side stream (on), or time both "
                         "once untimed and keep the faster (auto)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group (and run the return gather) even for one rank: "
                         "exercises the RCCL path on a one-GPU box (tests/test_gpu_rccl.py)")
    args = ap.parse_args()

    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus is not None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline runs first, before this process touches the GPU (its workers are forked)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)

    import torch
    dist = None
    # rehearsal: more ranks than visible GPUs (the 1-GPU dev box) -> all ranks on cuda:0, gloo on
    # host copies for the collectives; production: one rank per GPU, RCCL ("nccl") over xGMI
    rehearsal = world > 1 and torch.cuda.device_count() < world
    gpu = 0 if rehearsal else local
    coll_dev = "cpu" if rehearsal else torch.device("cuda", gpu)
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        if not launched:   # --force-dist without a launcher: a one-rank group on this host
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                free_port = sk.getsockname()[1]
            for k, v in (("WORLD_SIZE", "1"), ("RANK", "0"), ("LOCAL_RANK", "0"),
                         ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(free_port))):
                os.environ.setdefault(k, v)
        torch.cuda.set_device(gpu)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    strong = args.envs is None
    if strong:
        if args.global_envs % world:
            raise SystemExit(f"--global-envs {args.global_envs} does not split over {world} ranks")
        n_local = args.global_envs // world
    else:
        n_local = args.envs
    K, W = args.steps, args.warmup
    r = run_shard(args.env_id, n_local, rank, world, K, W, args.graph, dev, dist, coll_dev, args.overlap)
    weak = None
    if strong and world > 1 and not args.no_weak:   # secondary: 65536 envs per GPU
        w = run_shard(args.env_id, GLOBAL_ENVS, rank, world, K, W, args.graph, dev, dist, coll_dev, args.overlap)
        weak = {"envs_per_gpu": GLOBAL_ENVS, "global_envs": GLOBAL_ENVS * world, "value": w["inner"] / w["elapsed"],
                "ms_per_step": w["elapsed"] / K * 1e3, "kernel": w["env"].episode_kernel(),
                "kernel_ms": w["kern_ms"]}
        del w

    if rank == 0:
        env = r["env"]
        simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        line = {
            "metric": METRIC,
            "value": r["inner"] / r["elapsed"],
            "unit": "inner env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": r["elapsed"] / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reset(seed=0) -> env i seeded with its global index; MP params "
                    "default_rng(1234).standard_normal((N_global, 25), f32)",
            "config": {"workload": args.env_id, "global_envs": n_local * world, "envs_per_gpu": n_local,
                       "T": env.T, "launch": r["launch"],
                       "parallelism": f"env-shard x{world} (RCCL all_gather of the returns after every BB step)"
                       + (" [rehearsal: ranks share cuda:0, gloo]" if rehearsal else "")},
            "ranks_seen": dist.get_world_size() if dist is not None else 1,
            "backend": dist.get_backend() if dist is not None else None,
            "launcher": ("torch.distributed.run" + (" (spawned by bench.py --gpus)" if os.environ.get("FGX_BENCH_SPAWNED")
                                                     else "")) if launched else "single process",
            # per rank: [first global env, end, inner env steps in the timed region]
            "shards": r["shards"],
            # per rank: kernel time per BB step (HIP events around a kernel-only graph of K steps),
            # the timed BB step (episode + return all_gather, HIP events), their difference = the
            # per-step collective, the closing barrier (host, outside the value window) and the
            # number of return gathers inside the timed region (= steps when N > 1)
            "timing": {"kernel_ms_per_step_max": max(t["kernel_ms_per_step"] for t in r["per_rank"]),
                       "step_ms_max": max(t["step_ms"] for t in r["per_rank"]),
                       "exposed_collective_ms_per_step_max": max(t["exposed_collective_ms_per_step"]
                                                                 for t in r["per_rank"]),
                       "gather_ms_max": max((t["gather_ms"] for t in r["per_rank"] if t["gather_ms"] is not None),
                                            default=None),
                       "barrier_ms_max": max(t["barrier_ms"] for t in r["per_rank"]),
                       "gathers": r["gathers"],
                       "per_rank": r["per_rank"]},
            "roofline": roofline(args.env_id, env, n_local, r["kern_ms"], r["inner_local"], K, simds, lib_build_id()),
        }
        if r["schedule_trial"]:
            line["timing"]["schedule_trial"] = r["schedule_trial"]
        if r["capture_error"]:
            line["timing"]["capture_error"] = r["capture_error"]
        if weak is not None:
            line["weak_scaling"] = weak
        if world == 1 and env.T % 4 == 0:
            try:
                line["basis_gemm"] = basis_gemm(env, r["params"])
            except Exception as e:   # report, never fail the bench line on the side measurement
                line["basis_gemm"] = {"error": str(e)}
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
