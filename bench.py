"""Benchmark: 6DOF env-steps/s of the fused HIP step at N envs per GPU (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n ENVS_PER_GPU] [--model 6DOF|3DOF]
                    [--allgather] [--gather-leg | --no-gather-leg] [--no-sb3-legs] [--cpu-seconds S]

A "step" = one launch of the fused step kernel over all N envs of a GPU: action in,
RK4 rigid-body step + ground event + reward + done + obs + TimeLimit + auto-reset out.
Inputs (a pool of 8 pre-generated U(-1,1) action batches, seeded) are resident in HBM
before the timed region.

Multi-GPU: one process per GPU. ``--gpus N`` with N > 1 and no WORLD_SIZE in the environment
starts ``torch.distributed.run`` with N ranks as a CHILD process before anything touches the
GPU, and exits with its code (it fails loudly when fewer than N GPUs are visible); under
torchrun (WORLD_SIZE set) ``--gpus`` must equal WORLD_SIZE. Env shards [rank*N, (rank+1)*N)
with their own reset streams; the headline has no data-path collective. With more than one
rank the line also carries the step + all_gather leg (obs / reward / done
rows of every rank gathered each step, RCCL over xGMI), with the world size and backend the
communicator reports. Rehearsal on one GPU: RR_BENCH_ONE_DEVICE=1 puts every rank on cuda:0
and RR_BENCH_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU).

Prints ONE JSON line on rank 0 (see DESIGN.md §5 for every field).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic HBM bytes per env-step: read state+action+v0, write
# state+obs+reward+done.
BYTES_PER_STEP = {6: 56 + 12 + 4 + 56 + 56 + 4 + 1, 3: 28 + 8 + 4 + 28 + 28 + 4 + 1}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
POOL = 8
# --launch auto: direct launches (tools/libbench_timed.so) below this many timed steps, hipGraph
# replays from here on. Direct launches cost the host 3-4.8 us each against the kernel's ~4.2 us,
# so a run of them is host-paced at times: K = 20 at N = 65536 measured 5.5-6.6 us per step by
# the wall clock, one 20-launch graph replay 5.2-5.3 (round 4, profiles/r04/launch/)
AUTO_LOOP_MAX_K = 8
# warm-up of the n_sweep points: past the first episode ends, so that their K steps include the
# done path (terminal rows, auto-reset) at its steady rate
SWEEP_MIN_WARMUP = 100
REFERENCE_PY_STEP = {"6DOF": 569, "3DOF": 3396}  # SURVEY.md §6, survey container, 1 core


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--n", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--model", default="6DOF")
    ap.add_argument("--integrator", default="rk4")
    ap.add_argument("--allgather", action="store_true",
                    help="the headline itself is step rows + all_gather (ShardGather.step) every step")
    ap.add_argument("--gather-leg", action="store_true",
                    help="add the step + all_gather leg to the line at any world size (default: only when >1 rank)")
    ap.add_argument("--no-gather-leg", action="store_true")
    ap.add_argument("--monitor", action="store_true",
                    help="the drop-in default (RocketVecEnv monitor=True): Monitor running return kept per env "
                         "(read + written every step, +8 B per env-step); the headline runs without it")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--launch", default="auto", choices=["auto", "graph", "loop", "isolated"],
                    help="graph: K launches replayed from hipGraphs; loop: K direct launches of rr_step issued back "
                         "to back from C (tools/libbench_timed.so, action batch t mod 8 of the resident pool, the HIP "
                         "events recorded around them); auto: loop for K < %d, else graph (a graph replay carries "
                         "a fixed ~8 us preamble on the GPU timeline, a direct launch ~0.3 us more than a "
                         "graph-captured one: DESIGN.md section 5); isolated: one launch at a time, each between "
                         "its own pair of HIP events and followed by a host synchronize (kernel_us = the mean "
                         "isolated launch, the regime of a step between a policy's kernels)" % AUTO_LOOP_MAX_K)
    ap.add_argument("--graph-steps", type=int, default=1024,
                    help="env steps captured per hipGraph (each replay costs a fixed ~15-20 us on the GPU "
                         "timeline: 64 -> 4.34 us/step, 256 -> 4.25, 1024 -> 4.18 at N=65536)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sb3-legs", action="store_true",
                    help="skip the wall-clock legs through the Python boundary (RocketVecEnv.step with host and "
                         "device outputs, the single-env gym Rocket6DOF.step)")
    ap.add_argument("--sb3-steps", type=int, default=100)
    ap.add_argument("--n-sweep", default="4096,524288,4194304",
                    help="other envs-per-GPU points of the north star's N in {4k, 64k, 512k}, plus 4M (a ~1 GB "
                         "working set, 4x the 256 MB MALL: the true-HBM reading SURVEY.md 8d asks for), timed with "
                         "the same protocol (K steps after W warm-up, max over ranks) and reported in the line's "
                         "n_sweep (empty: none)")
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
    ap.add_argument("--no-ppo", action="store_true",
                    help="rollout mode: the collect only (no PPO update legs), e.g. for counter passes")
    ap.add_argument("--rollout-torch", action="store_true",
                    help="rollout policy / bootstrap / GAE as PyTorch ops instead of the fused HIP kernels")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# launching N ranks
# ---------------------------------------------------------------------------------------------
def launch_plan(gpus, environ):
    """("run", None): this process is the (only / a torchrun) rank; ("spawn", None): start
    torchrun with `gpus` ranks as a child; ("error", message) when --gpus contradicts WORLD_SIZE."""
    if gpus < 1:
        return "error", "--gpus must be >= 1"
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return ("spawn", None) if gpus > 1 else ("run", None)
    if int(ws) != gpus:
        return "error", ("bench.py --gpus %d but WORLD_SIZE=%s: the rank count and --gpus must agree" % (gpus, ws))
    return "run", None


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(gpus, argv):
    """torch.distributed.run with `gpus` ranks, started as a child process before this process
    has touched the GPU (torch.cuda.device_count() does not initialise it); returns its exit
    code. Fails loudly when the node shows fewer GPUs than ranks (unless RR_BENCH_ONE_DEVICE=1,
    the one-GPU rehearsal)."""
    import torch

    visible = torch.cuda.device_count()
    one_dev = os.environ.get("RR_BENCH_ONE_DEVICE") == "1"
    need = 1 if one_dev else gpus
    if visible < need:
        print("bench.py --gpus %d needs %d visible GPU(s), found %d (to rehearse N ranks on one GPU set "
              "RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo)" % (gpus, need, visible), file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------------------------
# the timed region
# ---------------------------------------------------------------------------------------------
class TimedLoop:
    """The event-timed direct-launch region: tools/libbench_timed.so (a benchmark-only helper,
    not the product ABI) issues K rr_step calls of the library behind a host-released gate
    kernel and records the two HIP events around them (tools/bench_timed.hip)."""

    def __init__(self, env):
        import ctypes

        from rl_rocket_amd import build as B

        path = B.BENCH_OUT
        if not os.path.exists(path):
            raise RuntimeError("%s is not built (python -m rl_rocket_amd.build)" % path)
        self.ct = ctypes
        self.lib = ctypes.CDLL(path)
        P = ctypes.c_void_p
        self.fn = self.lib.bt_step_repeat_timed
        self.fn.restype = ctypes.c_int
        self.fn.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, P, P, P, P, P, P, P]
        self.env = env
        self.rr_step = ctypes.cast(env.lib.rr_step, P)

    def call(self, actions, n_steps, events):
        """(function, arguments) of one timed call (prepared outside the timed region)."""
        ct, e = self.ct, self.env
        P = ct.c_void_p
        ev = [P(x.cuda_event) for x in events]
        if not all(x.value for x in ev):
            raise ValueError("record the events once before timing (they must exist)")
        ptr = lambda t: P(t.data_ptr()) if t is not None else None  # noqa: E731
        e._last_action = actions
        return self.fn, (self.rr_step, e._h, ptr(actions), actions.shape[0], e.num_envs * e.action_dim, int(n_steps),
                         ptr(e.obs), ptr(e.reward), ptr(e.done), ptr(e.truncated), ptr(e.terms), e._stream(),
                         ev[0], ev[1])


def per_rank_rows(dist, dt, kern_ms, K):
    """Every rank's own wall time and events figure of the timed region (at world > 1
    the line shows each rank, so a straggling rank is visible, not only the max over ranks)."""
    row = {"rank": dist.get_rank(), "wall_ms_per_step": dt / K * 1e3, "kernel_us": kern_ms * 1e3,
           "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}
    rows = [None] * dist.get_world_size()
    dist.all_gather_object(rows, row)
    return rows


def timed_region(args, env, pool, dev, dist, backend, launch, gather=None):
    """W untimed warm-up steps, then EXACTLY K steps bracketed by a barrier + synchronize on
    both sides; returns wall seconds (max over ranks), the per-launch device time by HIP
    events on the launch stream and, at world > 1, every rank's own pair of them."""
    import torch

    stream = torch.cuda.current_stream(dev)
    K = args.steps

    def one(k):
        if gather is not None:
            # the step writes obs / reward / done straight into the send rows (rr_step_rows),
            # then ONE all_gather: the global batch on every rank
            gather.step(env, pool[k % POOL])
        else:
            env.step(pool[k % POOL])

    use_loop = launch == "loop" and gather is None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if launch == "isolated":
        for k in range(args.warmup):
            one(k)
        torch.cuda.synchronize(dev)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(K):
            evs[k][0].record(stream)
            one(k)
            evs[k][1].record(stream)
            torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        if dist is not None:
            dist.barrier()
        per = sorted(a.elapsed_time(b) for a, b in evs)
        ranks = None
        if dist is not None:
            ranks = per_rank_rows(dist, dt, sum(per) / K, K)
            t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return {"dt": dt, "kern_ms": sum(per) / K, "use_graph": False, "use_loop": False, "gs": 0,
                "isolated_median_ms": per[K // 2], "isolated_min_ms": per[0], "per_rank": ranks}
    loop = TimedLoop(env) if use_loop else None
    if use_loop:
        ev0.record(stream)
        ev1.record(stream)
        fn, fargs = loop.call(pool, args.warmup, (ev0, ev1))
        rc = fn(*fargs)
        if rc != 0:
            raise RuntimeError("bt_step_repeat_timed (warm-up) failed: %d" % rc)
    else:
        for k in range(args.warmup):
            one(k)
    torch.cuda.synchronize(dev)

    # step + all_gather graphs need a capturable collective (RCCL); gloo is a host path
    use_graph = not args.no_graph and launch == "graph" and not (gather is not None and backend == "gloo")
    # exactly K steps: K // gs replays of a gs-launch graph (gs balanced so that K = 2000 is
    # 2 x 1000, not 1024 + 976) plus one graph of the K % gs remainder launches
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
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if use_loop:
        fn, fargs = loop.call(pool, K, (ev0, ev1))
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
    # each rank's own synchronize-to-synchronize time; the closing barrier (whose latency grows with
    # the rank count) stays outside it, and the max over ranks below covers any straggler
    dt = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    if use_loop and rc != 0:
        raise RuntimeError("bt_step_repeat_timed failed: %d" % rc)
    # device time per launch over the timed region (kernel + inter-kernel gap: an upper bound
    # on the kernel's own duration, so `achieved` is conservative)
    kern_ms = ev0.elapsed_time(ev1) / K
    ranks = None
    if dist is not None:  # every rank's own figures, then the max over ranks of the timed region
        ranks = per_rank_rows(dist, dt, kern_ms, K)
        t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return {"dt": dt, "kern_ms": kern_ms, "use_graph": use_graph, "use_loop": use_loop, "gs": gs,
            "per_rank": ranks}


# ---------------------------------------------------------------------------------------------
# rollout mode (BASELINE configs[4])
# ---------------------------------------------------------------------------------------------
# dense MFMA peaks, /opt/skills/guides/MI355X_MICROARCH.md: fp32 (v_mfma_f32_32x32x2_f32) 157.3
# TF; fp16 / bf16 ~2.5 PF (fp16x3 runs three fp16 MFMAs per product: priced at the fp16 peak)
ROLLOUT_PEAK_TFLOPS = {"fp32": 157.3, "fp16x3": 2500.0, "bf16": 2500.0}
HIDDEN = 64  # MlpPolicy net_arch [64, 64] (SB3 1.6 default for PPO)


def rollout_flops_per_env_step(ns, na):
    """Algorithmic FLOPs of the policy per env-step: the pi tower + action head and the vf tower
    + value head GEMMs of SB3's MlpPolicy (2 FLOP per multiply-add; tanh / sampling / the env
    step's VALU work not counted)."""
    tower = ns * HIDDEN + HIDDEN * HIDDEN
    return 2 * (tower + HIDDEN * na) + 2 * (tower + HIDDEN)


def rollout_bytes_per_env_step(ns, na, T):
    """Algorithmic HBM bytes per env-step of one collect: the rollout buffer slices written per step
    (obs, action, value, log-prob, start, reward, advantage, return) + per env and collect the
    state planes, v0 and counter read and written once, the last value / done / start and the last
    step's env outputs (obs, reward, done, truncated), spread over the T steps."""
    per_step = 4 * (ns + na + 6)
    per_collect = 2 * 4 * (ns + 2) + 3 * 4 + 4 * ns + 4 + 2
    return per_step + per_collect / T
def bench_rollout(args, dev, n, model, kw, dist=None, rank=0, world=1):
    """BASELINE configs[4]: N envs driving an on-device PPO rollout; the whole collect()
    (n_steps x [policy forward, Gaussian sample, env step, timeout bootstrap, buffer
    writes] + GAE) is one hipGraph; obs never leave HBM."""
    import torch

    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import MAX_EPISODE_STEPS
    from rl_rocket_amd.rollout import DeviceRollout, GraphedPPOUpdate, MlpActorCritic, ppo_update

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
    # The PPO update (SB3 1.6 PPO.train on the device-resident rollout, batch_size = N: n_steps
    # minibatches per epoch; one policy replica per GPU, minibatch gradients averaged over the
    # ranks with one all_reduce): eager PyTorch (one warm-up epoch, then one timed epoch) and the
    # minibatch step captured in one hipGraph (GraphedPPOUpdate) with PyTorch autograd and with
    # the rr_ppo_grad pipeline, then the end-to-end training iteration of configs[4]: one collect
    # + SB3's default n_epochs = 10 graphed epochs.
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5, capturable=True)
    grp = dist.group.WORLD if dist is not None else None

    def timed(fn):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t1, out

    update, stats, train = None, None, None
    if not args.no_ppo:
        ppo_update(pol, opt, ro, n_epochs=1, batch_size=n, group=grp)
        upd, stats = timed(lambda: ppo_update(pol, opt, ro, n_epochs=1, batch_size=n, group=grp))
        update = {"minibatches_per_epoch": args.rollout_steps, "batch_size": n, "eager_epoch_ms": upd * 1e3}
    if not args.no_ppo and (dist is None or dist.get_backend() == "nccl"):
        gt = GraphedPPOUpdate(pol, opt, ro, batch_size=n, group=grp, fused=False)
        gt.update(n_epochs=1)
        gupd, _ = timed(lambda: gt.update(n_epochs=3))
        update["graphed_epoch_ms"] = gupd * 1e3 / 3
        del gt
        # the loss + backward + clip + Adam from rr_ppo_update (fp32-MFMA HIP pipeline, chained
        # minibatches: three launches each) instead of autograd
        gu = GraphedPPOUpdate(pol, opt, ro, batch_size=n, group=grp, fused=True)
        gu.update(n_epochs=1)
        gupd, stats = timed(lambda: gu.update(n_epochs=10))
        update["fused_graphed_epoch_ms"] = gupd * 1e3 / 10
        update["fused_ms_per_minibatch"] = gupd * 1e3 / 10 / args.rollout_steps
        iters = 3

        def train_loop():
            for _ in range(iters):
                gu.prepare()  # the first epoch's permutation drawn beside the collect
                g.replay()
                gu.update(n_epochs=10)

        if dist is not None:
            dist.barrier()
        tt, _ = timed(train_loop)
        if dist is not None:
            t = torch.tensor([tt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tt = float(t.item())
        train = {"value": iters * args.rollout_steps * n * world / tt, "unit": "env-steps/s",
                 "ms_per_iteration": tt / iters * 1e3,
                 "what": "one training iteration = one collect (n_steps x N env-steps, one hipGraph) + 10 PPO epochs "
                         "of graphed minibatch updates (SB3 1.6 defaults: n_epochs 10), batch_size N, the whole "
                         "minibatch step (loss + backward + clip + Adam) by rr_ppo_update, chained; each epoch's "
                         "permutation drawn on a side stream beside the collect / the previous epoch"}
    env.close()
    # roofline of the collect kernel (rollout_step_kernel<..., MULTI = true>): the policy towers
    # are the contraction (fp32 MFMA in the default precision), so the bound is the MFMA peak;
    # algorithmic FLOPs = the two MlpPolicy towers' GEMMs (2 per multiply-add), algorithmic bytes =
    # the rollout buffer writes + the env state loaded / stored once per collect
    ns, na = env.state_dim, env.action_dim
    T = args.rollout_steps
    collect_s = e0.elapsed_time(e1) / reps * 1e-3
    flop = rollout_flops_per_env_step(ns, na) * n * T
    byt = rollout_bytes_per_env_step(ns, na, T) * n * T
    peak = ROLLOUT_PEAK_TFLOPS[args.policy_dtype]
    roof = {"bound": "mfma", "unit": "TFLOP/s", "peak": peak,
            "flops_per_env_step": rollout_flops_per_env_step(ns, na), "flops_per_launch": flop,
            "achieved_events": flop / collect_s / 1e12, "frac_events": flop / collect_s / 1e12 / peak,
            "hbm": {"bytes_per_env_step": rollout_bytes_per_env_step(ns, na, T), "bytes_per_launch": byt,
                    "achieved_GBs": byt / collect_s / 1e9, "frac": byt / collect_s / 1e9 / HBM_PEAK_GBS},
            "timing": "events: HIP events around the replays of the one-collect hipGraph (collect kernel + policy "
                      "pack + iteration counter); rocprof: the collect kernel's committed rocprofv3 kernel-trace mean "
                      "(same machine code)"}
    rp, rp_src = (None, "multi-rank run: committed 1-GPU traces are not quoted") if world > 1 else \
        stored_rollout_rocprof(model, n, T, args.policy_dtype)
    if rp is not None and not args.rollout_torch and ro.one_launch and not ro.per_step:
        roof.update(achieved=flop / (rp["mean_ns"] * 1e-9) / 1e12, rocprof_mean_us=rp["mean_ns"] / 1e3,
                    rocprof_source=rp_src, rocprof_median_of=rp.get("median_of"))
        roof["frac"] = roof["achieved"] / peak
        roof["frac_source"] = "rocprof"
    else:
        roof.update(achieved=roof["achieved_events"], frac=roof["frac_events"], frac_source="events",
                    rocprof_source=rp_src)
    return {
        "roofline": roof,
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
        "ppo_update": update, "ppo_stats": stats, "train_iteration": train,
    }


# ---------------------------------------------------------------------------------------------
# CPU baselines (rank 0, N = 1)
# ---------------------------------------------------------------------------------------------
def _cgroup_cpus():
    """CPUs of this process's cgroup quota (cpu.max "quota period"), or None when unlimited."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
        except (OSError, ValueError):
            continue
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    return None


def host_cores():
    """(threads the CPU legs use, how that count was found): the affinity mask, narrowed by
    the cgroup CPU quota and OMP_NUM_THREADS when they are set (the GPU box shows the whole
    machine in its affinity mask; its share is the quota / OMP_NUM_THREADS)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    src = {"affinity": aff}
    n = aff
    quota = _cgroup_cpus()
    if quota is not None:
        src["cgroup_quota"] = quota
        n = min(n, quota)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        src["OMP_NUM_THREADS"] = int(omp)
        n = min(n, int(omp))
    return max(1, n), src


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


def python_baseline(model, seconds):
    """the reference algorithm in the reference's language on ONE core — ONE
    env stepped from a Python loop by oracle/py_step.py (this repo's NumPy/SciPy restatement:
    a Python RHS under scipy.integrate.solve_ivp RK45 with the terminal ground event, then the
    reward, done and obs in NumPy; pinned to the reference's rows, tests/test_py_step.py)."""
    from oracle.py_step import run_episodes

    steps, busy = run_episodes(model, seconds)
    name = "6DOF" if model == 6 else "3DOF"
    return {"value": steps / busy, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "%d env-steps of ONE %s env from a Python loop, oracle/py_step.py (NumPy/SciPy restatement of "
                      "the reference's step(): solve_ivp RK45 + event, reward, done, obs; rocket_env.py:%d), %s ICs, "
                      "U(-1,1) actions, reset on done / TimeLimit 800, 1 thread"
                      % (steps, name, 690 if model == 6 else 150, "env_config" if model == 6 else "ctor-default")}


def cpu_baselines(model, seconds, cores):
    """cpu_baseline block of the bench line. Head: the north star's 'reference single-env CPU
    step()' — the NumPy/SciPy single-env restatement on one core (python_restatement_1core),
    then the C port of the same algorithm (one env per call from Python, batched on 1 core,
    batched on every host core of the box's share), the 3DOF single env of configs[0] in both
    forms, and the reference's own Python step() rates measured in the survey container (it
    cannot run on the GPU box)."""
    n_cores, src = cores
    py6 = python_baseline(model, seconds * 0.3)
    head = dict(py6)
    head["python_restatement_1core"] = py6
    head["c_port_single_env_1core"] = cpu_baseline(model, seconds * 0.15, n=1)
    head["batched_1core"] = cpu_baseline(model, seconds * 0.15)
    if n_cores > 1:
        head["all_cores"] = cpu_baseline(model, seconds * 0.15, nthreads=n_cores, n=8192)
        head["all_cores"]["cores_from"] = src
    if model == 6:
        head["configs0_3dof_python_restatement_1core"] = python_baseline(3, seconds * 0.1)
        head["configs0_3dof_single_env"] = cpu_baseline(3, seconds * 0.1, n=1)
    head["reference_python_step_survey"] = dict(REFERENCE_PY_STEP, unit="env-steps/s", cores=1,
                                                source="reference Rocket6DOF / Rocket step(), measured in the survey "
                                                       "container (SURVEY.md §6, BASELINE.md), not on this box")
    return head


# ---------------------------------------------------------------------------------------------
# wall-clock legs through the Python boundary (what SB3 calls)
# ---------------------------------------------------------------------------------------------
def _host_cpu():
    """(process CPU seconds, cgroup CPU-throttled microseconds or None, threads) — evidence for
    host-side stalls in the SB3-facing legs (a throttled cgroup stalls the stepping thread)."""
    t = os.times()
    thr = None
    for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            kv = dict(line.split() for line in open(path) if line.strip())
        except OSError:
            continue
        if "throttled_usec" in kv:
            thr = int(kv["throttled_usec"])
        elif "throttled_time" in kv:
            thr = int(kv["throttled_time"]) // 1000
        break
    threads = None
    try:
        threads = int([x for x in open("/proc/self/status") if x.startswith("Threads:")][0].split()[1])
    except (OSError, IndexError, ValueError):
        pass
    return t.user + t.system, thr, threads


def _host_delta(a, b, dt):
    return {"process_cpu_per_wall": round((b[0] - a[0]) / dt, 3),
            "cgroup_throttled_ms": None if a[1] is None or b[1] is None else round((b[1] - a[1]) / 1e3, 1),
            "threads": b[2]}


def sb3_collect_loop(dev, n, steps, rng):
    """Per step, what SB3 1.6 OnPolicyAlgorithm.collect_rollouts does with a VecEnv's outputs
    (the path main_6DOF.py:90-93's model.learn drives): np.clip of the policy's actions to the
    action space, env.step, _update_info_buffer (info.get("episode") / info.get("is_success")
    over every env's info) and the loop over every done flag that reads terminal_observation /
    TimeLimit.truncated. Wall clock; the split is measured in the same pass."""
    import collections

    import numpy as np
    import torch

    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS
    from rl_rocket_amd.vec_env import RocketVecEnv

    venv = RocketVecEnv(n, model="6DOF", device=dev, max_episode_steps=MAX_EPISODE_STEPS, monitor=True,
                        **ENV_CONFIG_6DOF)
    venv.reset()
    low, high = venv.action_space.low, venv.action_space.high
    pool = [rng.normal(0.0, 1.0, (n, 3)).astype(np.float32) for _ in range(POOL)]  # Gaussian policy samples
    ep_info_buffer = collections.deque(maxlen=100)
    ep_success_buffer = collections.deque(maxlen=100)
    split = {"clip": 0.0, "step": 0.0, "update_info_buffer": 0.0, "dones_loop": 0.0}

    def one(k, tm):
        t0 = time.perf_counter()
        clipped = np.clip(pool[k % POOL], low, high)
        t1 = time.perf_counter()
        _, _, dones, infos = venv.step(clipped)
        t2 = time.perf_counter()
        for idx, info in enumerate(infos):  # BaseAlgorithm._update_info_buffer
            maybe_ep_info = info.get("episode")
            maybe_is_success = info.get("is_success")
            if maybe_ep_info is not None:
                ep_info_buffer.extend([maybe_ep_info])
            if maybe_is_success is not None and dones[idx]:
                ep_success_buffer.append(maybe_is_success)
        t3 = time.perf_counter()
        n_boot = 0
        for idx, done in enumerate(dones):  # the timeout bootstrap's scan
            if done and infos[idx].get("terminal_observation") is not None and \
                    infos[idx].get("TimeLimit.truncated", False):
                n_boot += 1
        t4 = time.perf_counter()
        if tm:
            split["clip"] += t1 - t0
            split["step"] += t2 - t1
            split["update_info_buffer"] += t3 - t2
            split["dones_loop"] += t4 - t3
        return n_boot

    for k in range(100):  # the same warm-up as the other legs
        one(k, False)
    t0 = time.perf_counter()
    for k in range(steps):
        one(k, True)
    dt = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    venv.close()
    return {"value": n * steps / dt, "unit": "env-steps/s", "us_per_step": dt / steps * 1e6, "n_envs": n,
            "steps": steps, "split_us_per_step": {k: v / steps * 1e6 for k, v in split.items()},
            "episodes_seen": len(ep_info_buffer),
            "path": "SB3 1.6 collect_rollouts' per-step env work on RocketVecEnv(monitor=True) with numpy outputs: "
                    "np.clip(actions) + step + _update_info_buffer over all N infos + the done-flag loop "
                    "(terminal_observation / TimeLimit.truncated); the policy forward and the terminal-obs value "
                    "calls excluded"}


def sb3_legs(dev, n, steps):
    """env-steps/s through the drop-in surface, wall clock, Monitor on, random actions:
    RocketVecEnv.step with host (numpy) outputs — what SB3's DummyVecEnv.step_wait returns,
    replacing DummyVecEnv -> Monitor -> TimeLimit -> Rocket6DOF.step (rocket_env.py:690-719) — and
    with device_outputs=True (torch tensors left in HBM), each with its cost per step split into
    launch, kernel wait, D2H copies and Python infos; and the single-env gym shim
    Rocket6DOF.step (one launch + one sync per step) beside the reference's own 569 steps/s."""
    import numpy as np
    import torch

    from rl_rocket_amd.envs import Rocket6DOF
    from rl_rocket_amd.params import ENV_CONFIG_6DOF, MAX_EPISODE_STEPS
    from rl_rocket_amd.vec_env import RocketVecEnv

    WARM_SB3 = 100
    out = {}
    rng = np.random.default_rng(0)
    host_pool = [rng.uniform(-1, 1, (n, 3)).astype(np.float32) for _ in range(POOL)]

    def run(venv, acts, k0, count, host=True):
        n_done = 0
        for k in range(count):
            _, _, d, infos = venv.step(acts[(k0 + k) % POOL])
            if host:  # numpy flags (device flags are left alone: counting them would sync)
                n_done += int(d.sum())
        torch.cuda.synchronize(dev)
        return n_done

    # host outputs: numpy actions in, numpy obs / reward / done + lazy infos out
    venv = RocketVecEnv(n, model="6DOF", device=dev, max_episode_steps=MAX_EPISODE_STEPS, monitor=True,
                        **ENV_CONFIG_6DOF)
    venv.reset()
    # 100 warm-up steps: in the first ~100 steps after an env is created the host's synchronize
    # sporadically waits several ms while the device time of the step stays ~50 us (HIP events,
    # tools/probe_vecenv_host.py; profiles/r03/vh/): a region that starts earlier measures those
    run(venv, host_pool, 0, WARM_SB3)
    h0 = _host_cpu()
    t0 = time.perf_counter()
    n_done = run(venv, host_pool, WARM_SB3, steps)
    dt = time.perf_counter() - t0
    host = _host_delta(h0, _host_cpu(), dt)
    venv.timing = {}
    run(venv, host_pool, 0, steps)
    split = {k: v / steps * 1e6 for k, v in venv.timing.items()}
    venv.close()
    out["vecenv_host"] = {
        "value": n * steps / dt, "unit": "env-steps/s", "us_per_step": dt / steps * 1e6, "n_envs": n, "steps": steps,
        "done_per_step": n_done / steps, "host": host,
        "split_us_per_step": split,
        "split_note": "second pass with a synchronize after the launch: launch = action H2D + rr_step call (host), "
                      "kernel = remaining device time, d2h = obs / reward / done copies to numpy, infos = done list "
                      "(rr_fetch_done) + terminal_observation / TimeLimit.truncated / Monitor dicts of the done envs",
        "path": "RocketVecEnv(monitor=True).step(numpy actions) -> numpy obs/reward/done + lazy infos (SB3 VecEnv)"}

    # what stock SB3 1.6 does around that step (collect_rollouts, on_policy_algorithm.py): clip the
    # policy's actions, step, _update_info_buffer over ALL N infos, and the timeout-bootstrap loop
    # over every done flag reading terminal_observation / TimeLimit.truncated (the policy forward
    # and the value of the terminal obs are the policy's cost, not the env's: left out)
    out["sb3_collect_loop"] = sb3_collect_loop(dev, n, steps, rng)

    # device outputs: device actions in, device tensors out (obs stay in HBM); with Monitor (every
    # step's infos built two steps later) and without (nothing leaves HBM unless read). The same
    # warm-up (the first device-output steps also pay one-time pinned-buffer / allocator costs)
    pool = torch.rand((POOL, n, 3), device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 2 - 1
    for mon in (True, False):
        venv = RocketVecEnv(n, model="6DOF", device=dev, max_episode_steps=MAX_EPISODE_STEPS, monitor=mon,
                            device_outputs=True, **ENV_CONFIG_6DOF)
        venv.reset()
        run(venv, pool, 0, WARM_SB3, host=False)
        t0 = time.perf_counter()
        run(venv, pool, WARM_SB3, steps, host=False)
        dt = time.perf_counter() - t0
        venv.timing = {}
        run(venv, pool, 0, steps, host=False)
        split = {k: v / steps * 1e6 for k, v in venv.timing.items()}
        venv.close()
        out["vecenv_device" + ("" if mon else "_no_monitor")] = {
            "value": n * steps / dt, "unit": "env-steps/s", "us_per_step": dt / steps * 1e6, "n_envs": n,
            "steps": steps, "split_us_per_step": split,
            "split_note": "launch = rr_step + the done rows' terminal copy (host time of the async calls); infos = "
                          "the Monitor build of step t-2's infos (done-flag D2H, which waits for the GPU, + the done "
                          "rows' gather)" if mon else "launch = rr_step + the done rows' terminal copy; nothing else",
            "path": "RocketVecEnv(monitor=%s, device_outputs=True).step(device actions) -> device tensors + lazy "
                    "infos" % mon}

    # the single-env gym shim: one env, one launch + one packed D2H per step
    env = Rocket6DOF(device=dev, **ENV_CONFIG_6DOF)
    env.reset()
    a_pool = rng.uniform(-1, 1, (256, 3)).astype(np.float32)
    for k in range(20):
        if env.step(a_pool[k])[2]:
            env.reset()
    count, t0 = 0, time.perf_counter()
    while count < 3000 and time.perf_counter() - t0 < 3.0:
        if env.step(a_pool[count % 256])[2]:
            env.reset()
        count += 1
    dt = time.perf_counter() - t0
    env.close()
    out["single_env_gym"] = {
        "value": count / dt, "unit": "env-steps/s", "us_per_step": dt / count * 1e6, "steps": count,
        "vs_reference_python_step_survey": count / dt / REFERENCE_PY_STEP["6DOF"],
        "path": "rl_rocket_amd.envs.Rocket6DOF.step (gym API, N=1 kernel launch + sync per step, reset via gym "
                "0.21 seeding on the host)"}
    return out


# ---------------------------------------------------------------------------------------------
# committed evidence of the same kernel source (rocprofv3 PMC traffic, kernel-trace durations)
# ---------------------------------------------------------------------------------------------
_ISA = {}


def _isa_hashes():
    """ISA hash per kernel of the library this process runs (rl_rocket_amd.build.kernel_isa_hashes)."""
    if not _ISA:
        from rl_rocket_amd import build as B
        try:
            _ISA.update(B.kernel_isa_hashes(B.OUT))
        except Exception as e:  # noqa: BLE001 - tools missing: quote nothing
            _ISA["__error__"] = str(e)
    return _ISA


def launch_kind(launch):
    """'graph' / 'direct' / 'eager' of a bench line's config.launch string (or a stored trace's)."""
    launch = (launch or "").strip()
    if launch.startswith("graph"):
        return "graph"
    if launch.startswith("direct"):
        return "direct"
    return "eager"


def _stored(pattern, model, n, key, kernel_prefix=None, launch=None, upper=True):
    """The committed profile files matching `pattern` for this kernel and N whose kernel machine
    code (isa_hash of its kernel_name) is the code this process runs — and, with `launch`
    ('graph' / 'direct'), that were recorded with the same launch mode as the running command
    (a trace of direct launches does not describe graph replays: the tracer's per-dispatch cost
    differs). Of those, the median one by `key` in the conservative direction of that key
    (upper=True: the upper median, for a duration; upper=False: the lower median, for a byte count
    that would raise a bandwidth), never the best of two; the matching files are listed under
    `median_of`, the selection under `selection`. Else (None, reason)."""
    import glob

    prefix = kernel_prefix or ("step_kernel<%d," % model)
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", pattern % n), recursive=True))
    isa = _isa_hashes()
    stale, other_launch, match = None, None, []
    for path in hits:
        with open(path) as f:
            d = json.load(f)
        if not d.get("kernel", "").startswith(prefix):
            continue
        if not (d.get("isa_hash") and isa.get(d.get("kernel_name")) == d["isa_hash"]):
            stale = stale or os.path.relpath(path, ROOT)
        elif launch is not None and launch_kind(d.get("launch")) != launch:
            other_launch = other_launch or os.path.relpath(path, ROOT)
        else:
            match.append((d[key], os.path.relpath(path, ROOT), d))
    if match:
        match.sort(key=lambda m: m[0])
        v, src, d = match[len(match) // 2 if upper else (len(match) - 1) // 2]
        d = dict(d, median_of="%d files of this code%s: %s" % (
            len(match), "" if launch is None else " and launch mode (%s)" % launch,
            ", ".join("%s %.6g" % (m[1], m[0]) for m in match)),
            selection="%s median by %s of the committed files of this machine code%s" % (
                "upper" if upper else "lower", key, "" if launch is None else ", %s launches only" % launch))
        return d, src
    return None, ("no file measured on this kernel's machine code%s (other code: %s%s)%s"
                  % ("" if launch is None else " with %s launches" % launch, stale,
                     "" if other_launch is None else "; other launch mode: %s" % other_launch,
                     "; " + isa["__error__"] if "__error__" in isa else ""))


def stored_traffic(model, n):
    """Per-launch HBM bytes of the same kernel/config from the latest committed rocprofv3 PMC
    passes (tools/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE), only if they were measured on
    THIS kernel's machine code (same ISA hash): the lower median; else (None, reason)."""
    d, src = _stored("pmc_traffic_n%d.json", model, n, "traffic_bytes", upper=False)
    return (d["traffic_bytes"], src) if d else (None, src)


def stored_rocprof(model, n, steps, launch=None):
    """The step kernel's rocprofv3 kernel-trace mean of the same protocol (tools/rocprof_step.py:
    a --kernel-trace --stats run of this bench command, committed under profiles/), only if it
    was measured on THIS kernel's machine code and, with `launch`, with the same launch mode;
    the upper median; else (None, reason)."""
    return _stored("rocprof_step_k%d_n%%d.json" % steps, model, n, "mean_ns", launch=launch)


def stored_exact_fp64(n):
    """fp64 VALU issue rate of the exact-mode kernel at this N (profiles/**/exact_counters_n<N>.json
    measured on the machine code this process runs): the upper median of the matching files."""
    import glob

    isa = _isa_hashes()
    match = []
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "exact_counters_n%d.json" % n),
                                 recursive=True)):
        with open(path) as f:
            d = json.load(f)
        if d.get("fp64") and d.get("isa_hash") and isa.get(d.get("kernel_name")) == d["isa_hash"]:
            match.append((d["fp64"]["achieved_tflops"], os.path.relpath(path, ROOT), d))
    if not match:
        return {"source": "no exact-mode counters of this machine code at N = %d" % n}
    match.sort(key=lambda m: m[0])
    v, src, d = match[len(match) // 2]
    return {"bound": "fp64 VALU", "achieved": v, "peak": d["fp64"]["peak_tflops"], "unit": "TFLOP/s",
            "frac": d["fp64"]["frac"], "kernel_us": d["kernel_trace"]["mean_us"], "kernel": d["kernel_name"],
            "what": d["fp64"]["what"], "source": src}


def stored_rollout_rocprof(model, n, T, dtype):
    """The collect kernel's committed rocprofv3 kernel-trace mean (tools/rocprof_step.py on a
    `bench.py --mode rollout` run) measured on this kernel's machine code; else (None, reason)."""
    return _stored("rocprof_rollout_n%%d_t%d_%s.json" % (T, dtype), model, n, "mean_ns",
                   kernel_prefix="rollout_step_kernel<%d," % model)


def gather_leg_result(args, env, pool, dev, dist, backend, launch, n, world, K):
    """The step + all_gather leg (reported separately from the step alone)."""
    from rl_rocket_amd.dist import ShardGather

    g = ShardGather(n, env.state_dim, dev)
    greg = timed_region(args, env, pool, dev, dist, backend, "graph" if launch in ("loop", "isolated") else launch, g)
    return {
        "value": n * world * K / greg["dt"], "unit": "env-steps/s", "ms_per_step": greg["dt"] / K * 1e3,
        "device_us_per_step": greg["kern_ms"] * 1e3, "per_rank": greg.get("per_rank"),
        "world_size": dist.get_world_size(), "backend": dist.get_backend(),
        "bytes_per_rank_per_step": g.n_pad * (env.state_dim + 2) * 4,
        "launch": "graph" if greg["use_graph"] else "eager (gloo stages through the host)",
        "what": "rr_step_rows into the send rows + ONE all_gather_into_tensor of [N][state_dim+2] fp32 rows "
                "(obs, reward, done) per step, the global batch on every rank (ShardGather.step)"}


def main():
    args = parse()
    plan, msg = launch_plan(args.gpus, os.environ)
    if plan == "error":
        print(msg, file=sys.stderr, flush=True)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    import numpy as np  # noqa: F401
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
    gather_leg = args.mode == "step" and not args.allgather and not args.no_gather_leg and (world > 1 or args.gather_leg)
    dist = None
    if world == 1 and (args.allgather or gather_leg):  # step + gather on one GPU (a rehearsal of the collective)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.allgather or gather_leg:
        import datetime

        import torch.distributed as dist
        # a rank that dies must not leave the others waiting in a collective for the default 10 min
        tmo = datetime.timedelta(seconds=int(os.environ.get("RR_BENCH_PG_TIMEOUT", "180")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        world = dist.get_world_size()

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
    launch = args.launch
    if launch == "auto":
        launch = "loop" if args.steps < AUTO_LOOP_MAX_K and not args.allgather else "graph"
    gather = None
    if args.allgather:
        from rl_rocket_amd.dist import ShardGather
        gather = ShardGather(n, env.state_dim, dev)

    # ---- the headline timed region ----
    reg = timed_region(args, env, pool, dev, dist, backend, launch, gather)
    K, dt, kern_ms = args.steps, reg["dt"], reg["kern_ms"]
    value = n * world * K / dt
    bytes_env = BYTES_PER_STEP[model] + (8 if args.monitor else 0)  # + Monitor return plane read / write
    bytes_launch = bytes_env * n
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    achieved_wall = bytes_launch / (dt / K) / 1e9
    headline_cfg = not (args.monitor or args.allgather or args.integrator != "rk4" or launch == "isolated")
    if headline_cfg:
        traffic, traffic_src = stored_traffic(model, n)
        rp, rp_src = stored_rocprof(model, n, K, launch="graph" if reg["use_graph"] else
                                    "direct" if reg["use_loop"] else "eager")
    else:
        traffic, traffic_src = None, "PMC traffic files cover the headline configuration (RK4, no Monitor, no gather)"
        rp, rp_src = None, "rocprofv3 files cover the headline configuration"
    if args.integrator == "euler":
        parity = ("explicit Euler of the reference RHS (BASELINE configs[1] 'Euler integrator'): within 1e-6 of the "
                  "oracle's fp64 Euler restatement (oracle/rocket_oracle.c euler_step; tests/test_gpu_parity.py::"
                  "test_euler_vs_oracle_euler); a declared NON-PARITY mode against the reference's RK45 step (30-130x "
                  "its 1e-5 bar, tests/test_gpu_envs.py::test_euler_mode_is_declared_non_parity)")
    elif args.integrator == "dopri5":
        parity = ("exact mode: fp64 scipy RK45 + brentq restated, <= 4.4e-9 floored-relative vs the reference's "
                  "rows (tests/test_gpu_exact.py)")
    else:
        parity = ("fp32 RK4 + Hermite ground event, <= 1e-5 floored-relative vs the reference's rows and the "
                  "oracle (tests/test_gpu_parity.py)")
    rocprof = None
    if rp is not None:
        rocprof = {"mean_us": rp["mean_ns"] / 1e3, "frac": bytes_launch / (rp["mean_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS,
                   "calls": rp["calls"], "events_us_same_run": rp.get("events_kernel_us"), "source": rp_src,
                   "launch": rp.get("launch"), "median_of": rp.get("median_of"), "selection": rp.get("selection")}
    # `frac` is the profile-evidenced figure where a committed rocprofv3 kernel trace of this
    # command on this kernel's machine code exists (one GPU only: a stored 1-GPU trace does not
    # describe the ranks of a multi-GPU run), the live HIP-event figure otherwise
    stored_1gpu = None
    if rocprof is not None and world > 1:
        stored_1gpu, rocprof = rocprof, None
    frac_events = achieved / HBM_PEAK_GBS
    if rocprof is not None:
        achieved_line, frac_line = bytes_launch / (rp["mean_ns"] * 1e-9) / 1e9, rocprof["frac"]
        frac_source = "rocprof: %s (mean kernel-trace duration of this command, %d dispatches; %s)" % (
            rp_src, rp["calls"], rp.get("selection"))
        # the live HIP-event figure against the committed trace: the tracer adds its per-dispatch
        # completion handling (~0.5 us at N = 65 536), so events normally read a few to
        # ~15 % above it; outside [0.85, 1.30] the committed figure does not describe this run
        ratio = frac_events / rocprof["frac"]
        rocprof["events_over_rocprof"] = ratio
        if not 0.85 <= ratio <= 1.30:
            rocprof["warning"] = ("the live events figure (%.3f) and the committed rocprofv3 figure (%.3f) differ by "
                                  "more than the tracer's overhead explains" % (frac_events, rocprof["frac"]))
    else:
        achieved_line, frac_line = achieved, frac_events
        frac_source = "events: HIP events on the launch stream around the K launches of this run" + \
            ("" if world == 1 else " (world %d: committed 1-GPU traces are not quoted)" % world)
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
        "dtype": "fp64" if args.integrator == "dopri5" else "fp32",
        "parity": parity,
        "data": "synthetic: ICs ~ U(init_space of configuration_file.env_config), actions ~ U(-1,1) seeded pool of %d "
                "batches resident in HBM" % POOL,
        "config": {"workload": "Rocket%s N=%d per GPU, %s fused step+reward+TimeLimit(800)+auto-reset, %s"
                               % ("6DOF" if model == 6 else "3DOF", n, args.integrator.upper(),
                                  "step rows + all_gather of obs/reward/done each step" if args.allgather else
                                  "no data-path collective") + (", Monitor returns" if args.monitor else ""),
                   "envs_per_gpu": n, "global_envs": n * world, "integrator": args.integrator,
                   "graph_steps": reg["gs"] if reg["use_graph"] else 0, "launch": "graph" if reg["use_graph"] else
                   ("direct: tools/libbench_timed.so (K rr_step calls)" if reg["use_loop"] else
                    "isolated: one rr_step between two HIP events + synchronize per step" if launch == "isolated" else
                    "rr_step per step"),
                   "parallelism": "env-sharded x%d" % world,
                   "world_size": dist.get_world_size() if dist is not None else 1,
                   "backend": dist.get_backend() if dist is not None else None},
        "roofline": {"bound": "hbm", "achieved": achieved_line, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": frac_line, "frac_source": frac_source,
                     "achieved_events": achieved, "frac_events": frac_events,
                     "frac_wall": achieved_wall / HBM_PEAK_GBS,
                     "frac_rocprof": rocprof["frac"] if rocprof else None,
                     "rocprof": rocprof if rocprof else (
                         {"source": rp_src} if stored_1gpu is None else
                         {"stored_1gpu_profile": stored_1gpu,
                          "note": "a committed single-GPU rocprofv3 trace of this kernel; not a measurement of this "
                                  "%d-rank run, so frac_rocprof is null and frac is the events figure" % world}),
                     "traffic": traffic, "traffic_unit": "B/launch",
                     "traffic_source": traffic_src,
                     "kernel": "step_kernel<%d,%s>" % (model, args.integrator.upper()),
                     "kernel_us": kern_ms * 1e3,
                     "timing": "frac_events: HIP events on the launch stream around the K launches of the timed region" +
                               (" (recorded by tools/libbench_timed.so; the first 2 launches are queued behind a "
                                "host-released gate kernel so the host's submission stays ahead)"
                                if reg["use_loop"] else " (around the hipGraph replays)") +
                               (" (each step = rr_step_rows + the all_gather, so kernel_us includes the "
                                "collective)" if gather is not None else "") +
                               "; frac_wall: the same bytes over the wall-clock ms_per_step; frac_rocprof: over the "
                               "rocprofv3 kernel-trace mean of this command on this kernel's machine code (committed "
                               "under profiles/); frac = frac_rocprof where that trace exists (one GPU), else "
                               "frac_events",
                     "bytes_per_launch": bytes_launch,
                     "bytes_per_env_step": bytes_env},
    }

    if reg.get("per_rank"):
        walls = [r["wall_ms_per_step"] for r in reg["per_rank"]]
        result["per_rank"] = reg["per_rank"]
        result["per_rank_wall_max_over_min"] = max(walls) / min(walls)
    if args.integrator == "dopri5" and world == 1:
        # the exact mode is fp64 VALU work, not HBM-bound: its issue rate against the fp64 vector
        # peak from the committed counters of the same N and machine code (tools/exact_counters.py)
        result["roofline_fp64"] = stored_exact_fp64(n)

    # ---- the step + all_gather leg (reported separately from the step alone) ----
    if launch == "isolated":
        result["roofline"]["isolated_median_us"] = reg["isolated_median_ms"] * 1e3
        result["roofline"]["isolated_min_us"] = reg["isolated_min_ms"] * 1e3
    if gather_leg:
        # failures are reported in the line, never at the expense of the step-only headline (the
        # process group's timeout bounds any wait on a rank that failed first)
        try:
            result["allgather"] = gather_leg_result(args, env, pool, dev, dist, backend, launch, n, world, K)
        except Exception as e:  # noqa: BLE001
            result["allgather"] = {"error": "%s: %s" % (type(e).__name__, e)}
    env.close()
    sweep = [int(x) for x in args.n_sweep.split(",") if x.strip()] if args.mode == "step" and not args.allgather else []
    if sweep:
        result["n_sweep"] = []
        for n_i in sweep:
            e_i = RocketBatch(n_i, model=model, device=dev, max_episode_steps=MAX_EPISODE_STEPS, auto_reset=True,
                              episode_stats=args.monitor, integrator=args.integrator, env_id_offset=rank * n_i, **kw)
            e_i.reset()
            g_i = torch.Generator(device=dev)
            g_i.manual_seed(42 + rank)
            p_i = torch.rand((POOL, n_i, e_i.action_dim), device=dev, generator=g_i) * 2 - 1
            # steady state: the timed steps come after the first episode ends (from step ~30 on,
            # ~1.5 % of the envs end an episode per step; tools/phase_probe.py). Before them no lane
            # takes the done path, which at N >= 524 288 costs 5-25 % (terminal rows, auto-reset)
            a_i = argparse.Namespace(**vars(args))
            a_i.warmup = max(args.warmup, SWEEP_MIN_WARMUP)
            r_i = timed_region(a_i, e_i, p_i, dev, dist, backend, launch)
            b_i = bytes_env * n_i
            result["n_sweep"].append({
                "envs_per_gpu": n_i, "warmup": a_i.warmup, "global_envs": n_i * world, "value": n_i * world * K / r_i["dt"],
                "ms_per_step": r_i["dt"] / K * 1e3, "kernel_us": r_i["kern_ms"] * 1e3,
                "frac": b_i / (r_i["kern_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "frac_wall": b_i / (r_i["dt"] / K) / 1e9 / HBM_PEAK_GBS})
            if r_i.get("per_rank"):
                walls = [r["wall_ms_per_step"] for r in r_i["per_rank"]]
                result["n_sweep"][-1]["per_rank"] = r_i["per_rank"]
                result["n_sweep"][-1]["per_rank_wall_max_over_min"] = max(walls) / min(walls)
            e_i.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baselines(model, args.cpu_seconds, host_cores())
    if rank == 0 and world == 1 and model == 6 and not args.no_sb3_legs and args.integrator == "rk4":
        result["sb3_legs"] = sb3_legs(dev, n, args.sb3_steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
