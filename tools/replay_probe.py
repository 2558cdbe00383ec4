"""Where the per-replay cost of a short hipGraph goes (driver protocol K = 20).

    python tools/replay_probe.py [--k 20] [--reps 7] [--n 65536]

Captures K rr_step launches of the bench workload into one hipGraph and times one replay
several ways (median over --reps replays, µs per launch):

  outer_null     torch events on the current (null) stream around graph.replay() — bench.py
  outer_stream   the same on a non-default stream (capture and replay there)
  upload         hipGraphUpload of the exec before the timed replays, then outer_null
  nofence        outer events created with hipEventDisableSystemFence
  inner          event-record captured INSIDE the graph (hipEventRecordWithFlags with
                 hipEventRecordExternal before the first and after the last step launch)
  nodes          event-record NODES added to the captured graph (hipGraphAddEventRecordNode:
                 one before the root, one after the leaf): the K launches without the
                 replay's preamble; nodes_outer = outer events around the same replays

The HIP calls go through torch's own libamdhip64 (ctypes), on the streams torch hands out.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
HIP_EVENT_RECORD_EXTERNAL = 0x01


def hip():
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    for name in ("hipEventCreateWithFlags", "hipEventRecordWithFlags", "hipEventRecord", "hipEventElapsedTime",
                 "hipGraphUpload", "hipEventSynchronize", "hipEventDestroy", "hipGraphGetNodes", "hipGraphGetRootNodes",
                 "hipGraphNodeGetDependentNodes", "hipGraphAddEventRecordNode", "hipGraphAddDependencies"):
        getattr(lib, name).restype = ctypes.c_int
    return lib


def check(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: hipError %d" % (what, rc))


class RawEvent:
    def __init__(self, lib, flags=0):
        self.lib, self.h = lib, ctypes.c_void_p()
        check(lib.hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(flags)), "hipEventCreateWithFlags")

    def record(self, stream, flags=0):
        check(self.lib.hipEventRecordWithFlags(self.h, ctypes.c_void_p(stream.cuda_stream), ctypes.c_uint(flags)),
              "hipEventRecordWithFlags")

    def ms_to(self, other):
        out = ctypes.c_float()
        check(self.lib.hipEventElapsedTime(ctypes.byref(out), self.h, other.h), "hipEventElapsedTime")
        return out.value


def add_event_nodes(lib, graph, ev0, ev1):
    """ev0 -> root ... leaf -> ev1 on a captured linear graph (raw hipGraph_t)."""
    g = ctypes.c_void_p(graph)
    n = ctypes.c_size_t(0)
    check(lib.hipGraphGetRootNodes(g, None, ctypes.byref(n)), "hipGraphGetRootNodes")
    roots = (ctypes.c_void_p * n.value)()
    check(lib.hipGraphGetRootNodes(g, roots, ctypes.byref(n)), "hipGraphGetRootNodes")
    m = ctypes.c_size_t(0)
    check(lib.hipGraphGetNodes(g, None, ctypes.byref(m)), "hipGraphGetNodes")
    nodes = (ctypes.c_void_p * m.value)()
    check(lib.hipGraphGetNodes(g, nodes, ctypes.byref(m)), "hipGraphGetNodes")
    leaves = []
    for nd in nodes:
        k = ctypes.c_size_t(0)
        check(lib.hipGraphNodeGetDependentNodes(ctypes.c_void_p(nd), None, ctypes.byref(k)), "GetDependentNodes")
        if k.value == 0:
            leaves.append(nd)
    e0 = ctypes.c_void_p()
    check(lib.hipGraphAddEventRecordNode(ctypes.byref(e0), g, None, ctypes.c_size_t(0), ev0.h), "AddEventRecordNode")
    for r in roots:
        check(lib.hipGraphAddDependencies(g, ctypes.byref(e0), ctypes.byref(ctypes.c_void_p(r)), ctypes.c_size_t(1)),
              "hipGraphAddDependencies")
    lv = (ctypes.c_void_p * len(leaves))(*leaves)
    e1 = ctypes.c_void_p()
    check(lib.hipGraphAddEventRecordNode(ctypes.byref(e1), g, lv, ctypes.c_size_t(len(leaves)), ev1.h),
          "AddEventRecordNode")
    return len(roots), len(leaves), m.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--external", action="store_true", help="also try hipEventRecordExternal inside the capture")
    a = ap.parse_args()
    from rl_rocket_amd.batch import RocketBatch
    from rl_rocket_amd.params import ENV_CONFIG_6DOF

    lib = hip()
    dev = torch.device("cuda", 0)
    env = RocketBatch(a.n, model=6, device=dev, max_episode_steps=800, auto_reset=True, episode_stats=False,
                      **ENV_CONFIG_6DOF)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    pool = torch.rand((8, a.n, 3), device=dev, generator=g) * 2 - 1
    for k in range(5):
        env.step(pool[k % 8])
    torch.cuda.synchronize()

    def capture(stream, inner=None):
        gr = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        with torch.cuda.stream(cap):
            with torch.cuda.graph(gr, stream=cap):
                if inner:
                    inner[0].record(cap, HIP_EVENT_RECORD_EXTERNAL)
                for k in range(a.k):
                    env.step(pool[k % 8])
                if inner:
                    inner[1].record(cap, HIP_EVENT_RECORD_EXTERNAL)
        stream.wait_stream(cap)
        torch.cuda.synchronize()
        gr.replay()
        torch.cuda.synchronize()
        return gr

    def timed(gr, stream, ev_flags=0, inner=None):
        out = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = RawEvent(lib, ev_flags), RawEvent(lib, ev_flags)
            with torch.cuda.stream(stream):
                e0.record(stream)
                gr.replay()
                e1.record(stream)
            torch.cuda.synchronize()
            out.append((inner[0].ms_to(inner[1]) if inner else e0.ms_to(e1)) * 1e3 / a.k)
        return out

    null = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    res = {}
    gr = capture(null)
    res["outer_null"] = timed(gr, null)
    res["nofence"] = timed(gr, null, HIP_EVENT_DISABLE_SYSTEM_FENCE)
    check(lib.hipGraphUpload(ctypes.c_void_p(gr.raw_cuda_graph_exec()), ctypes.c_void_p(null.cuda_stream)),
          "hipGraphUpload")
    torch.cuda.synchronize()
    res["upload"] = timed(gr, null)
    gs = capture(side)
    res["outer_stream"] = timed(gs, side)
    if a.external:  # refused on this ROCm build: hipErrorInvalidValue inside the capture
        try:
            inner = (RawEvent(lib), RawEvent(lib))
            gi = capture(null, inner)
            res["inner"] = timed(gi, null, inner=inner)
        except RuntimeError as e:
            res["inner_error"] = str(e)
    try:
        inner = (RawEvent(lib), RawEvent(lib))
        gk = torch.cuda.CUDAGraph(keep_graph=True)
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(null)
        with torch.cuda.stream(cap):
            with torch.cuda.graph(gk, stream=cap):
                for k in range(a.k):
                    env.step(pool[k % 8])
        null.wait_stream(cap)
        torch.cuda.synchronize()
        res["nodes_shape"] = add_event_nodes(lib, gk.raw_cuda_graph(), inner[0], inner[1])
        gk.instantiate()
        gk.replay()
        torch.cuda.synchronize()
        res["nodes"] = timed(gk, null, inner=inner)
        res["nodes_outer"] = timed(gk, null)
    except RuntimeError as e:
        res["nodes_error"] = str(e)
    res["outer_null_again"] = timed(gr, null)
    print(json.dumps({"k": a.k, "n": a.n, "us_per_launch": {
        k: ({"median": statistics.median(v), "runs": [round(x, 4) for x in v]} if isinstance(v, list) else v)
        for k, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
