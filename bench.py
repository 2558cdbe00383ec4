"""Benchmark: 6DOF env-steps/s of the fused HIP step at N envs per GPU (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n ENVS_PER_GPU] [--model 6DOF|3DOF]
                    [--allgather] [--no-graph] [--cpu-seconds S]

A "step" = one launch of the fused step kernel over all N envs of a GPU: action in,
RK4 rigid-body step + ground event + reward + done + obs + TimeLimit + auto-reset out.
Inputs (a pool of 8 pre-generated U(-1,1) action batches, seeded) are resident in HBM
before the timed region. Multi-GPU: one process per GPU (torchrun), env shards
[rank*N, (rank+1)*N) with their own RNG streams; no data-path collective unless
--allgather (RCCL all_gather of obs/reward/done after every step).

Prints ONE JSON line on rank 0 (see DESIGN.md §5 for every field).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic HBM bytes per env-step: read state+action+v0, write
# state+obs+reward+done.
BYTES_PER_STEP = {6: 56 + 12 + 4 + 56 + 56 + 4 + 1, 3: 28 + 8 + 4 + 28 + 28 + 4 + 1}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
POOL = 8
# --launch auto: direct launches (rr_step_repeat_timed) below this many timed steps, hipGraph
# replays from here on (crossover of the ~8 us per-replay preamble against ~0.3 us per direct
# launch, measured at N = 65536: DESIGN.md section 5)
AUTO_LOOP_MAX_K = 32


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--n", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--model", default="6DOF")
    ap.add_argument("--integrator", default="rk4")
    ap.add_argument("--allgather", action="store_true")
    ap.add_argument("--monitor", action="store_true",
                    help="the drop-in default (RocketVecEnv monitor=True): Monitor running return kept per env "
                         "(read + written every step, +8 B per env-step); the headline runs without it")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--launch", default="auto", choices=["auto", "graph", "loop"],
                    help="graph: K launches replayed from hipGraphs; loop: one rr_step_repeat_timed call (K direct "
                         "launches issued back to back from C, action batch t mod 8 of the resident pool, the HIP "
                         "events recorded by the call around them); auto: loop for K < %d, else graph (a graph "
                         "replay carries a fixed ~8 us preamble on the GPU timeline, a direct launch ~0.3 us more "
                         "than a graph-captured one: DESIGN.md section 5)" % AUTO_LOOP_MAX_K)
    ap.add_argument("--graph-steps", type=int, default=1024,
                    help="env steps captured per hipGraph (each replay costs a fixed ~15-20 us on the GPU "
                         "timeline: 64 -> 4.34 us/step, 256 -> 4.25, 1024 -> 4.18 at N=65536)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default="step", choices=["step", "rollout"],
                    help="step: the fused env step (headline); rollout: on-device PPO rollout "
                         "collection (MlpPolicy 64x64 forward + sample + env step + buffer), BASELINE configs[4]")
    ap.add_argument("--rollout-steps", type=int, default=16)
    ap.add_argument("--policy-dtype", default="fp32", choices=["fp32", "fp16x3", "bf16"],
                    help="rollout mode: fused policy towers on fp32 MFMA (SB3-exact, default), split-fp16 MFMA "
                         "(fp16x3: operands as fp16 hi + lo, three MFMAs per k step, fp32-level accuracy) or bf16 "
                         "MFMA with fp32 accumulation (opt-in)")
    ap.add_argument("--rollout-two-launch", action="store_true",
                    help="rollout mode: rr_policy_act + rr_step per step instead of the one-launch rr_rollout_collect")
    ap.add_argument("--rollout-per-step", action="store_true",
                    help="rollout mode: one rr_rollout_step launch per step (+ bootstrap + GAE launches) instead "
                         "of the whole collect in one rr_rollout_collect launch")
    ap.add_argument("--rollout-torch", action="store_true",
                    help="rollout policy / bootstrap / GAE as PyTorch ops instead of the fused HIP kernels")
    return ap.parse_args()


def bench_rollout(args, dev, n, model, kw, dist=None, rank=0, world=1):
    """BASELINE configs[4]: N envs driving an on-device PPO rollout; the whole collect()
    (n_steps x [policy forward, Gaussian sample, env step, timeout bootstrap, buffer
    writes] + GAE) is one hipGraph; obs never leave HBM."""
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import MAX_EPISODE_STEPS
    from rl_rocket_amd.rollout import DeviceRollout, MlpActorCritic, ppo_update

    torch.manual_seed(42)
    env = RocketBatch(n, model=model, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=False, integrator=args.integrator, env_id_offset=rank * n, **kw)
    pol = MlpActorCritic(env.state_dim, env.action_dim).to(dev)
    fused = not args.rollout_torch
    ro = DeviceRollout(env, pol, n_steps=args.rollout_steps, fused=fused, policy_dtype=args.policy_dtype,
                       one_launch=fused and not args.rollout_two_launch and args.integrator != "dopri5",
                       per_step=args.rollout_per_step)
    for _ in range(3):
        ro.collect()
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            ro.collect()
    torch.cuda.current_stream(dev).wait_stream(s)
    g.replay()
    torch.cuda.synchronize(dev)
    reps = max(2, args.steps // args.rollout_steps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if dist is not None:  # max over ranks of the timed region
        t = torch.tensor([dt], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    steps = reps * args.rollout_steps
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    # one policy replica per GPU: minibatch gradients averaged over the ranks (one all_reduce)
    stats = ppo_update(pol, opt, ro, n_epochs=1, batch_size=n, group=dist.group.WORLD if dist is not None else None)
    torch.cuda.synchronize(dev)
    upd = time.perf_counter() - t1
    env.close()
    return {
        "metric": "env-steps/sec of on-device PPO rollout collection (%s, N=%d per GPU)"
                  % ("6DOF" if model == 6 else "3DOF", n),
        "value": n * world * steps / dt, "unit": "env-steps/s", "n_gpus": world, "steps": steps, "warmup": 3 * args.rollout_steps,
        "ms_per_step": dt / steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": {"fp32": "fp32", "fp16x3": "fp32 env, split-fp16 MFMA policy towers (fp16 hi + lo operands, fp32 "
                  "accumulate)", "bf16": "fp32 env, bf16-MFMA policy towers (fp32 accumulate)"}[args.policy_dtype],
        "data": "synthetic ICs (env_config init_space), actions from a random-init MlpPolicy",
        "config": {"workload": "Rocket6DOF N=%d, MlpPolicy(64x64 tanh) forward + Gaussian sample + fused step "
                               "+ timeout bootstrap + rollout buffer + GAE, n_steps=%d per hipGraph"
                               % (n, args.rollout_steps), "envs_per_gpu": n,
                   "policy_path": "PyTorch ops" if args.rollout_torch else
                   ("one launch per collect: rr_rollout_collect (n_steps x [policy on %s MFMA + env step] + GAE)"
                    if ro.one_launch and not ro.per_step else
                    "one launch per step: rr_rollout_step (policy on %s MFMA + env step)" if ro.one_launch else
                    "two launches per step: rr_policy_act (%s MFMA) + rr_step") % args.policy_dtype},
        "gpu_ms_per_collect": e0.elapsed_time(e1) / reps,
        "ppo_epoch_ms": upd * 1e3, "ppo_stats": stats,
    }


def host_cores():
    """CPU threads this process may use (the GPU box shows the whole machine in
    os.cpu_count(); its share is the affinity mask / OMP_NUM_THREADS)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else max(1, min(n, 16))


def cpu_baseline(model, seconds, seed=0, nthreads=1, n=1024):
    """The CPU oracle (faithful scipy-RK45 restatement in C) stepping a bounded sample of
    the same workload: envs from the same init_space, U(-1,1) actions, auto-reset on done,
    TimeLimit 800. n = 1: ONE env per call from a Python loop, the shape of the reference's
    single-env ``Rocket6DOF.step()`` (rocket_env.py:690, 150); n > 1: the batched port,
    `nthreads` OpenMP threads over the env batch (SURVEY.md §8d baselines (i) and (ii))."""
    import numpy as np

    from oracle import oracle as O

    kw = O.ENV_CONFIG_6DOF if model == 6 else O.DEFAULTS_3DOF
    cfg = O.make_cfg(model, **kw)
    ns = 14 if model == 6 else 7
    na = 3 if model == 6 else 2
    lo_ic = (np.float32(kw["IC"]) - np.float32(kw["ICRange"]) / 2).astype(np.float32)
    hi_ic = (np.float32(kw["IC"]) + np.float32(kw["ICRange"]) / 2).astype(np.float32)
    rng = np.random.default_rng(seed)

    def sample(k):
        ic = rng.uniform(lo_ic, hi_ic, (k, ns)).astype(np.float32)
        if model == 6:
            ic[:, 6:10] /= np.linalg.norm(ic[:, 6:10], axis=1, keepdims=True)
        return ic

    ic = sample(n)
    s = ic.astype(np.float64)
    el = np.zeros(n, np.int64)
    t = np.zeros(n)
    steps = 0
    busy = 0.0
    while busy < seconds:
        a = rng.uniform(-1, 1, (n, na)).astype(np.float32)
        t0 = time.perf_counter()
        out = O.step(cfg, ic, t, s, a, nthreads=nthreads)
        busy += time.perf_counter() - t0
        steps += n
        s = out["state_out"]
        t = np.round(t + cfg.dt, 3)
        el += 1
        d = out["done"] | (el >= 800)
        if d.any():
            k = int(d.sum())
            ic[d] = sample(k)
            s[d] = ic[d]
            el[d] = 0
            t[d] = 0
    name = "6DOF" if model == 6 else "3DOF"
    if n == 1:
        what = ("%d env-steps of ONE %s env, one oracle call per step from a Python loop (the shape of the "
                "reference's single-env step(), rocket_env.py:%d), env_config ICs, U(-1,1) actions, auto-reset, "
                "TimeLimit 800" % (steps, name, 690 if model == 6 else 150))
    else:
        what = ("%d env-steps of %s (%d envs x %d steps per call, batched oracle ro_step_batch), env_config ICs, "
                "U(-1,1) actions, auto-reset, TimeLimit 800" % (steps, name, n, steps // n))
    return {"value": steps / busy, "unit": "env-steps/s", "cores": nthreads, "kind": "port",
            "sample": what + ", %d thread(s), oracle/librocket_oracle.so (scipy RK45 + brentq restated in C)" % nthreads}


def cpu_baselines(model, seconds, cores):
    """cpu_baseline block of the bench line: the single-env leg (the north star's 'reference
    single-env CPU step()'), the batched port on 1 core and on all host cores, the 3DOF single
    env of configs[0], and the reference's own Python step() rates measured in the survey
    container (it cannot run on the GPU box)."""
    head = cpu_baseline(model, seconds * 0.35, n=1)
    head["batched_1core"] = cpu_baseline(model, seconds * 0.25)
    if cores > 1:
        head["all_cores"] = cpu_baseline(model, seconds * 0.2, nthreads=cores, n=8192)
    if model == 6:
        head["configs0_3dof_single_env"] = cpu_baseline(3, seconds * 0.2, n=1)
    head["reference_python_step_survey"] = {"6DOF": 569, "3DOF": 3396, "unit": "env-steps/s", "cores": 1,
                                            "source": "reference Rocket6DOF / Rocket step(), measured in the survey "
                                                      "container (SURVEY.md §6, BASELINE.md), not on this box"}
    return head


def stored_traffic(model, n):
    """Per-launch HBM bytes of the same kernel/config from the latest committed rocprofv3 PMC
    passes (tools/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE), only if they were measured on
    THIS kernel code (same rl_rocket_amd.build.source_hash); else (None, reason)."""
    import glob

    from rl_rocket_amd.build import source_hash

    want = source_hash()
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "pmc_traffic_n%d.json" % n), recursive=True),
                  key=os.path.getmtime)
    stale = None
    for path in reversed(hits):
        d = json.load(open(path))
        if not d.get("kernel", "").startswith("step_kernel<%d," % model):
            continue
        if d.get("source_hash") == want:
            return d["traffic_bytes"], os.path.relpath(path, ROOT)
        stale = stale or os.path.relpath(path, ROOT)
    return None, ("no PMC traffic file for kernel source %s (latest, other source: %s)" % (want, stale))


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for the N > 1 path on a one-GPU box (not used by the driver's runs):
    # RR_BENCH_ONE_DEVICE=1 puts every rank on cuda:0, RR_BENCH_BACKEND=gloo replaces RCCL
    # (RCCL refuses two ranks on one GPU). Default: one GPU per rank over RCCL.
    if os.environ.get("RR_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("RR_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world == 1 and args.allgather:  # step + gather path on one GPU (a rehearsal of the collective)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.allgather:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS, parse_model

    model = parse_model(args.model)
    kw = ENV_CONFIG_6DOF if model == 6 else {}
    n = args.n
    if args.mode == "rollout":
        res = bench_rollout(args, dev, n, model, kw, dist=dist, rank=rank, world=world)
        if rank == 0:
            print(json.dumps(res), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    env = RocketBatch(n, model=model, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                      episode_stats=args.monitor, integrator=args.integrator, env_id_offset=rank * n, **kw)
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    pool = torch.rand((POOL, n, env.action_dim), device=dev, generator=gen) * 2 - 1
    gather = None
    if args.allgather and dist is not None:
        from rl_rocket_amd.dist import ShardGather
        gather = ShardGather(n, env.state_dim, dev)

    def one(k):
        if gather is not None:
            # the step writes obs / reward / done straight into the send rows (rr_step_rows),
            # then ONE RCCL all_gather over xGMI: the global batch on every rank
            gather.step(env, pool[k % POOL])
        else:
            env.step(pool[k % POOL])

    stream = torch.cuda.current_stream(dev)
    launch = args.launch
    if launch == "auto":
        launch = "loop" if args.steps < AUTO_LOOP_MAX_K and not args.allgather else "graph"
    use_loop = launch == "loop" and not args.allgather
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if use_loop:
        # the same call as the timed region (its launch block is written once, here), and the
        # two timing events created so that the C call can record them
        ev0.record(stream)
        ev1.record(stream)
        env.step_repeat(pool, args.warmup, events=(ev0, ev1))
    else:
        for k in range(args.warmup):
            one(k)
    torch.cuda.synchronize(dev)

    # ---- timed region: exactly K steps (hipGraph replays) ----
    # step + all_gather graphs need a capturable collective (RCCL); gloo is a host path
    use_graph = not args.no_graph and launch == "graph" and not (gather is not None and backend == "gloo")
    # exactly K steps: K // gs replays of a gs-launch graph (gs balanced so that K = 2000 is
    # 2 x 1000, not 1024 + 976) plus one graph of the K % gs remainder launches
    K = args.steps
    gs = max(1, -(-K // max(1, -(-K // max(1, args.graph_steps)))))
    rem = K % gs

    def capture(n_launch):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(stream)
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for k in range(n_launch):
                    one(k)
        stream.wait_stream(s)
        torch.cuda.synchronize(dev)
        g.replay()  # warm the graph
        torch.cuda.synchronize(dev)
        return g

    if use_graph:
        graph = capture(gs)
        graph_rem = capture(rem) if rem else None
    # Device time of the K launches: HIP events on the launch stream around the replays. It
    # includes hipGraphLaunch's fixed preamble on the GPU timeline (~6-8 us per replay, so
    # +0.3-0.4 us per step at the driver's K = 20); event-record nodes inside the graph, which
    # would exclude it, are refused by torch on ROCm ("External events are disallowed").
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if use_loop:
        fn, fargs = env.step_repeat_call(pool, K, (ev0, ev1))
    t0 = time.perf_counter()
    if use_loop:
        # K direct launches from one C call, which records the two HIP events on the launch
        # stream right before the first and right after the last launch
        rc = fn(*fargs)
    else:
        ev0.record(stream)  # HIP events on the stream the step kernels are launched on
        if use_graph:
            for _ in range(K // gs):
                graph.replay()
            if graph_rem is not None:
                graph_rem.replay()
        else:
            for k in range(K):
                one(k)
        ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if use_loop:
        from rl_rocket_amd import _lib
        _lib.check(rc, "rr_step_repeat_timed")
    # device time per launch over the timed region (kernel + inter-kernel gap inside the
    # graph: an upper bound on the kernel's own duration, so `achieved` is conservative).
    # (Events recorded with hipEventReleaseToDevice instead of torch's system-scope release
    # read the same at K = 20: 4.58 vs 4.56 us per launch, r02o.)
    kern_ms = ev0.elapsed_time(ev1) / K
    if dist is not None:  # max over ranks of the timed region
        t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    value = n * world * K / dt
    bytes_env = BYTES_PER_STEP[model] + (8 if args.monitor else 0)  # + Monitor return plane read / write
    bytes_launch = bytes_env * n
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    if args.monitor or args.allgather or args.integrator != "rk4":
        traffic, traffic_src = None, "PMC traffic files cover the headline configuration (RK4, no Monitor, no gather)"
    else:
        traffic, traffic_src = stored_traffic(model, n)
    result = {
        "metric": "env-steps/sec (%s, N=%d per GPU)" % ("6DOF" if model == 6 else "3DOF", n),
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": dt / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: ICs ~ U(init_space of configuration_file.env_config), actions ~ U(-1,1) seeded pool of %d "
                "batches resident in HBM" % POOL,
        "config": {"workload": "Rocket%s N=%d per GPU, %s fused step+reward+TimeLimit(800)+auto-reset, %s"
                               % ("6DOF" if model == 6 else "3DOF", n, args.integrator.upper(),
                                  "step rows + RCCL all_gather of obs/reward/done each step" if args.allgather else
                                  "no data-path collective") + (", Monitor returns" if args.monitor else ""),
                   "envs_per_gpu": n, "global_envs": n * world, "integrator": args.integrator,
                   "graph_steps": gs if use_graph else 0, "launch": "graph" if use_graph else
                   ("direct: rr_step_repeat_timed" if use_loop else "rr_step per step"),
                   "parallelism": "env-sharded x%d" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "B/launch",
                     "traffic_source": traffic_src,
                     "kernel": "step_kernel<%d,%s>" % (model, args.integrator.upper()),
                     "kernel_us": kern_ms * 1e3,
                     "timing": "HIP events on the launch stream around the K launches of the timed region" +
                               (" (recorded by rr_step_repeat_timed itself; the first 2 launches are queued "
                                "behind a host-released gate kernel so the host's submission stays ahead)"
                                if use_loop else " (around the hipGraph replays)") +
                               (" (each step = rr_step_rows + the RCCL all_gather, so kernel_us includes the "
                                "collective)" if gather is not None else ""),
                     "bytes_per_launch": bytes_launch,
                     "bytes_per_env_step": bytes_env},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baselines(model, args.cpu_seconds, host_cores())
    env.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
