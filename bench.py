"""Benchmark: inner env-steps/s of fancy_ProMP/LongSimpleReacher-v0 black-box steps on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--envs ENVS_PER_GPU]
For N > 1 launch with torch.distributed.run (one process per GPU); env shards are independent
(weak scaling: ENVS_PER_GPU envs per rank, seeds = global env index), RCCL only gathers the
final episode returns.  Prints ONE JSON line on rank 0.

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
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "inner env-steps/sec, ProMP 5-link Reacher, N=65536 envs at 1/2/4/8 MI355X"
WORKLOAD = "fancy_ProMP/LongSimpleReacher-v0"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_VEC_PEAK_TF = 78.6    # MI355X FP64 vector peak (spec; half the 157.3 TF FP32 vector peak)


FP32_VEC_PEAK_TF = 157.3   # MI355X_MICROARCH.md: Peak FP32 (vector)
CLOCK_GHZ = 2.4            # MI355X peak engine clock
# cycles per VALU instruction a single wave sustains with 8 independent f64 fma chains, and the
# SIMD with >= 4 waves (profiles/r01_valu_rates.jsonl): k_episode runs one wave per SIMD
SINGLE_WAVE_CYCLES = 6.12
SIMD_CYCLES = 4.68
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_k_episode.json")
PMC_ISSUE = os.path.join(ROOT, "profiles", "r01_pmc_issue_k_episode.json")


def pmc_issue(env_id, n_envs):
    """Issue-side PMC of the metric kernel (committed rocprofv3 passes): VALUBusy and VALU
    instructions per inner step."""
    if env_id != WORKLOAD or n_envs != 65536:
        return None
    try:
        with open(PMC_ISSUE) as f:
            d = json.load(f)
        c, per = d["counters_per_dispatch"], d["per_wave_sample"]
        return {"valu_busy_pct": c["VALUBusy"], "valu_lane_util_pct": c["VALUUtilization"],
                "valu_instr_per_inner_step_per_wave": per["SQ_INSTS_VALU"],
                "f64_add_mul_fma_per_inner_step_per_wave": per["SQ_INSTS_VALU_ADD_F64"]
                + per["SQ_INSTS_VALU_MUL_F64"] + per["SQ_INSTS_VALU_FMA_F64"],
                "source": "profiles/r01_pmc_issue_k_episode.json"}
    except (OSError, ValueError, KeyError):
        return None


def episode_flops_per_step(env):
    """Algorithmic flops of one inner env step of k_episode (PD controller, torque env).
    f32: basis contraction (2 flop per fma) + velocity difference/division;
    f64: PD (5 per dof), clip (0), Euler (4 per dof), control cost (2 per dof - 1), return (1)."""
    n, nb = env.dof, 5
    f32 = n * (2 * nb + 3)
    f64 = n * 5 + n * 4 + (2 * n - 1) + 1
    return f32, f64


def pmc_traffic(env_id, n_envs):
    """HBM bytes per k_episode launch from the committed rocprofv3 PMC pass (FETCH_SIZE x2 per the
    gfx950 half-count correction + WRITE_SIZE, KiB -> B), if it was taken on this workload."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        if d.get("workload") == env_id and int(d.get("envs")) == n_envs:
            return float(d["traffic_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def episode_bytes_per_env(env):
    """Algorithmic HBM bytes of one k_episode launch per env (info_level 0, autoreset on)."""
    n, P, out = env.dof, env.n_params, env.out_dim
    hole = 0 if env._eng.cfg.env_kind == 0 else 3 * 8      # SimpleReacher kernels skip hole / aux
    state = 2 * n * 8 + 2 * 8 + hole + 3 * 4 + 5 * 8       # q, qd, goal, [hole], steps/plans/flags, rng
    reads = P * 4 + state
    writes = state + 2 * out * 4 + 8 + 1 + 1 + 4           # state, obs, final_obs, ret, term, trunc, len
    return reads + writes


def basis_gemm(env, params, reps=10):
    """The MP basis x weights contraction as its own launch (BlackBoxWrapper.get_trajectory ->
    fgx_trajectory -> k_traj_mfma, v_mfma_f32_32x32x2_f32 with K = 8): time per launch from HIP
    events around a graph replay of `reps` launches, MFMA utilisation against the f32 matrix peak
    and the HBM rate of its [N, T, dof] f32 outputs."""
    N, T, n = env.num_envs, env.T, env.dof
    pos = torch.empty((N, T, n), dtype=torch.float32, device=params.device)
    vel = torch.empty_like(pos)
    lib, h = env._eng.lib, env._eng.h
    import ctypes
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
    flops = 2 * 2 * 8 * N * n * T                 # two K = 8 GEMMs (positions, next positions)
    out_bytes = 2 * 4 * N * T * n + 4 * N * env.n_params
    return {"kernel": "k_traj_mfma", "us": t * 1e6, "mfma_tflops": flops / t / 1e12,
            "peak_tflops": FP32_VEC_PEAK_TF, "mfma_frac": flops / t / 1e12 / FP32_VEC_PEAK_TF,
            "hbm_GBps": out_bytes / t / 1e9, "hbm_frac": out_bytes / t / 1e9 / HBM_PEAK_GBS,
            "note": "K = 8 (5 basis + zero pad): arithmetic intensity 2 flop/B, bound by the output "
                    "write; the fused k_episode evaluates the same contraction in registers instead"}


def cpu_baseline(seconds=12.0, cores=None):
    """The oracle port (structure-matched per-env Python loop of the reference) on host cores."""
    import multiprocessing as mp_
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = cores or max(1, min(16, aff))
    ctx = mp_.get_context("fork")
    with ctx.Pool(cores) as pool:
        t0 = time.perf_counter()
        res = pool.map(_cpu_worker, [(i, seconds) for i in range(cores)])
        wall = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    return dict(value=steps / wall, unit="inner env-steps/s", cores=cores, kind="port",
                sample=f"oracle/port.py per-env loop (f32 ProMP contraction + PD + 200 substeps with the "
                       f"reference's per-step numpy ops incl. its 2 self-collision checks + autoreset), "
                       f"{WORKLOAD}, {cores} processes x ~{seconds:.0f}s, {steps} inner steps; "
                       f"os.cpu_count()={os.cpu_count()}, affinity={aff}")


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--env-id", default=WORKLOAD)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="launch the K steps eagerly instead of replaying them as one HIP graph")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # rehearsal: more ranks than visible GPUs (the 1-GPU dev box) -> all ranks on cuda:0, gloo on
    # host copies for the collectives; production: one rank per GPU, RCCL ("nccl") over xGMI
    rehearsal = world > 1 and torch.cuda.device_count() < world
    gpu = 0 if rehearsal else local
    coll_dev = "cpu" if rehearsal else torch.device("cuda", gpu)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    import fancy_gym_crowd_amd as fgx
    from fancy_gym_crowd_amd import shard
    N = args.envs
    lo, _ = shard.shard_range(N, rank, world)
    env = fgx.make(args.env_id, num_envs=N, device=dev, seed_offset=lo)
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
    acc = torch.zeros(1, dtype=torch.int64, device=dev)   # device counter of inner env steps

    for _ in range(args.warmup):
        env.step_into(params, obs, ret, te, tr, tl, fobs)
    torch.cuda.synchronize()
    acc.zero_()

    K = args.steps
    graph = None
    if args.graph:
        # the K BB-step launches captured once in a HIP graph (the same kernels on the same state;
        # removes the per-launch host round trip between dependent steps)
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for k in range(K):
                    env.step_into(params, obs, ret, te, tr, tl, fobs, inner_steps=acc)
            torch.cuda.synchronize()
        except Exception as e:   # capture unsupported: time the eager launches instead
            print(f"[bench] graph capture failed ({e}); timing eager launches", file=sys.stderr)
            graph = None
    acc.zero_()
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        ev0[0].record()
        graph.replay()
        ev1[0].record()
    else:
        for k in range(K):
            ev0[k].record()
            env.step_into(params, obs, ret, te, tr, tl, fobs, inner_steps=acc)
            ev1[k].record()
    if dist is not None:   # final episode-return gather over RCCL/xGMI (the path's only exchange)
        all_ret = shard.gather_returns(ret.to(coll_dev))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    inner_local = int(acc.item())
    if graph is not None:   # HIP events around the replay on the launch stream: mean per BB step
        kern_ms = ev0[0].elapsed_time(ev1[0]) / K
    else:
        kern_ms = float(np.mean([ev0[k].elapsed_time(ev1[k]) for k in range(K)]))
    if dist is not None:
        elapsed = shard.max_over_ranks(elapsed, coll_dev)
        inner = shard.sum_over_ranks(inner_local, coll_dev)
        assert all_ret.numel() == N * world
    else:
        inner = inner_local

    if rank == 0:
        value = inner / elapsed
        f32f, f64f = episode_flops_per_step(env)
        steps_per_s_kernel = (inner_local / K) / (kern_ms * 1e-3)
        valu = {"f32_tflops": f32f * steps_per_s_kernel / 1e12, "f64_tflops": f64f * steps_per_s_kernel / 1e12,
                "peak_f32_tflops": FP32_VEC_PEAK_TF, "peak_f64_tflops": FP64_VEC_PEAK_TF,
                "frac": f32f * steps_per_s_kernel / 1e12 / FP32_VEC_PEAK_TF
                + f64f * steps_per_s_kernel / 1e12 / FP64_VEC_PEAK_TF,
                "pmc": pmc_issue(args.env_id, N)}
        if valu["pmc"] is not None:   # issue rate: VALU instructions per SIMD over the kernel time
            instr = valu["pmc"]["valu_instr_per_inner_step_per_wave"] * (inner_local / K) / 64.0
            simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
            cyc = kern_ms * 1e-3 * CLOCK_GHZ * 1e9 / (instr / simds)
            valu["issue"] = {"cycles_per_valu_instr_per_simd": cyc,
                             "single_wave_floor_cycles": SINGLE_WAVE_CYCLES, "simd_floor_cycles": SIMD_CYCLES,
                             "frac_of_single_wave_issue": SINGLE_WAVE_CYCLES / cyc,
                             "frac_of_simd_issue": SIMD_CYCLES / cyc,
                             "note": "one wave (64 envs) per SIMD at 65536 envs: the single-wave issue rate "
                                     "is the ceiling (DESIGN.md 4.3)"}
        bpe = episode_bytes_per_env(env)
        achieved = bpe * N / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "inner env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reset(seed=0) -> env i seeded with its global index; MP params "
                    "default_rng(1234).standard_normal((N_global, 25), f32)",
            "config": {"workload": args.env_id, "envs_per_gpu": N, "global_envs": N * world, "T": env.T,
                       "launch": "hip graph of the K steps" if graph is not None else "eager",
                       "parallelism": f"env-shard x{world} (RCCL all_gather of returns only)"
                       + (" [rehearsal: ranks share cuda:0, gloo]" if rehearsal else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(args.env_id, N),
                         "kernel": env.episode_kernel(), "kernel_ms": kern_ms, "bytes_per_env": bpe,
                         "bytes_per_inner_step": bpe * N / (inner_local / K),
                         "note": "state lives in registers for all T substeps: the kernel is VALU-issue "
                                 "bound (see valu); per-substep HBM design would need 242 B/step",
                         "valu": valu},
        }
        if world == 1 and env.T % 4 == 0:
            try:
                line["basis_gemm"] = basis_gemm(env, params)
            except Exception as e:   # report, never fail the bench line on the side measurement
                line["basis_gemm"] = {"error": str(e)}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
