"""The C-ABI library loads on a CPU-only host and exports exactly what
include/rocket_hip.h declares; the ctypes mirrors match the C struct layouts."""
import ctypes
import os
import re
import subprocess

import pytest

from rl_rocket_amd import _lib

HEADER = _lib.HEADER


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_bound_symbols():
    assert _declared_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in _declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r"\bT (rr_[a-z0-9_]+)", out))
    assert exported == set(_declared_functions())
    assert lib.rr_abi_version() == _lib.ABI_VERSION


def test_invalid_arguments_fail_cleanly_without_gpu():
    lib = _lib.load()
    p = _lib.RrParams()
    p.model = 5
    p.dt = 0.1
    h = ctypes.c_void_p()
    assert lib.rr_create(ctypes.byref(h), ctypes.byref(p), 16, 0, 0) == _lib.RR_EINVAL
    assert b"model" in lib.rr_last_error()
    p.model = 6
    p.integrator = 7
    assert lib.rr_create(ctypes.byref(h), ctypes.byref(p), 16, 0, 0) == _lib.RR_EINVAL
    p.integrator = 0
    p.max_episode_steps = 70000
    assert lib.rr_create(ctypes.byref(h), ctypes.byref(p), 16, 0, 0) == _lib.RR_EINVAL
    p.max_episode_steps = 800
    assert lib.rr_create(ctypes.byref(h), ctypes.byref(p), 0, 0, 0) == _lib.RR_EINVAL
    # the largest batch: n * (state_dim + 3) * 4 B within 32-bit buffer offsets (tests/test_gpu_maxsize.py)
    assert lib.rr_create(ctypes.byref(h), ctypes.byref(p), 0xFFFFFFFF // 68 + 1, 0, 0) == _lib.RR_EINVAL
    assert b"32-bit" in lib.rr_last_error()
    for bad in (0x40, 0x40000000, 0x80000000):  # the high bits are the kernels' internal mode word
        p.flags = 0x1 | bad
        assert lib.rr_create(ctypes.byref(h), ctypes.byref(p), 16, 0, 0) == _lib.RR_EINVAL
        assert b"flag" in lib.rr_last_error()
    p.flags = 0x1
    assert lib.rr_step(None, None, None, None, None, None, None, None) == _lib.RR_EINVAL
    assert lib.rr_destroy(None) == 0
    assert lib.rr_num_envs(None) == -1
    # rollout entry points: argument errors come back as codes before any HIP call
    assert lib.rr_rollout_step(None, None, 0, 0, None, 0, 0.99, *([None] * 12)) == _lib.RR_EINVAL
    assert lib.rr_rollout_collect(None, None, 0, 0, None, 16, 0.99, 0.95, *([None] * 17)) == _lib.RR_EINVAL
    assert b"rr_rollout_collect" in lib.rr_last_error()
    assert lib.rr_gae(0, 16, None, None, None, None, None, 0.99, 0.95, None, None, None) == _lib.RR_EINVAL


def _c_layout(struct, fields):
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"rocket_hip.h\"\nint main(void){\n"
    src += 'printf("%%zu\\n", sizeof(%s));\n' % struct
    for f in fields:
        src += 'printf("%%zu\\n", offsetof(%s, %s));\n' % (struct, f)
    src += "return 0;}\n"
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"), "rr_layout_%d" % os.getpid())
    os.makedirs(d, exist_ok=True)
    c = os.path.join(d, "l.c")
    open(c, "w").write(src)
    exe = os.path.join(d, "l")
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe])
    vals = [int(x) for x in subprocess.check_output([exe]).split()]
    return vals[0], vals[1:]


@pytest.mark.parametrize("cls,cname", [(_lib.RrParams, "rr_params"), (_lib.RrBuffers, "rr_buffers")])
def test_ctypes_struct_layout_matches_header(cls, cname):
    names = [f[0] for f in cls._fields_]
    size, offs = _c_layout(cname, names)
    assert ctypes.sizeof(cls) == size
    assert [getattr(cls, n).offset for n in names] == offs


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.RocketHipError, match="no CPU fallback"):
        _lib.load()


def _ptrs(k, null_at=None):
    """A host array of k fake non-null device pointers (never dereferenced: every call below is
    refused before it launches), with an optional null entry."""
    arr = (ctypes.c_void_p * k)(*[0x10000 + 0x1000 * i for i in range(k)])
    if null_at is not None:
        arr[null_at] = None
    return arr


def test_abi_8_to_12_entry_points_refuse_bad_arguments_before_any_hip_call():
    """Every entry point added in ABI 8-12 (rr_gather_rows, rr_copy_terminal, rr_step_rows,
    rr_host_alloc / rr_host_free, rr_ppo_grad, rr_clip_adam, rr_ppo_update, their workspace sizes,
    the rr_policy_* and rollout calls) returns RR_EINVAL with a message naming itself for null handles, null or
    inconsistent arguments and bad sizes — without touching HIP (this host has no GPU; tools/
    sanitize.sh runs this test under ASan + UBSan). Valid host-only calls (layout / workspace
    sizes) return the documented values."""
    lib = _lib.load()
    E = _lib.RR_EINVAL
    V = ctypes.c_void_p
    fake = V(0x10000)

    def refused(rc, name):
        assert rc == E, (name, rc)
        assert name.encode() in lib.rr_last_error(), (name, lib.rr_last_error())

    # env-handle calls
    refused(lib.rr_gather_rows(None, fake, fake, fake, fake, fake, 16, *([None] * 5), None), "rr_gather_rows")
    refused(lib.rr_gather_rows(fake, None, None, None, None, None, 16, *([None] * 5), None), "rr_gather_rows")
    refused(lib.rr_copy_terminal(None, fake, fake, fake, None), "rr_copy_terminal")
    refused(lib.rr_step_rows(None, fake, fake, None, None, None), "rr_step_rows")
    refused(lib.rr_step_repeat(None, fake, 1, 1, fake, fake, fake, None, None, None), "rr_step_repeat")
    refused(lib.rr_fetch_done(None, 16, None, None, None, None, None), "rr_fetch_done")
    refused(lib.rr_seed(None, 1, None), "rr_seed")
    refused(lib.rr_reset(None, None, None, None), "rr_reset")
    refused(lib.rr_set_state(None, fake, None, None, None), "rr_set_state")
    refused(lib.rr_get_state(None, None, None, None, None), "rr_get_state")
    refused(lib.rr_set_state64(None, fake, None, None, None), "rr_set_state64")
    refused(lib.rr_get_state64(None, None, None, None, None), "rr_get_state64")
    refused(lib.rr_get_aux(None, None, None, None), "rr_get_aux")
    refused(lib.rr_set_aux(None, None, None, None), "rr_set_aux")
    refused(lib.rr_get_buffers(None, None), "rr_get_buffers")
    assert lib.rr_counter_bits(None) == E
    # pinned host memory
    out = V()
    refused(lib.rr_host_alloc(ctypes.byref(out), 0), "rr_host_alloc")
    refused(lib.rr_host_alloc(ctypes.byref(out), -5), "rr_host_alloc")
    refused(lib.rr_host_alloc(None, 64), "rr_host_alloc")
    assert lib.rr_host_free(None) == 0
    # policy: layout sizes (host only), pack / act / bootstrap refusals
    off = (ctypes.c_int64 * 12)()
    for ns, na in ((14, 3), (7, 2)):
        for prec in (0, 1, 2):
            size = lib.rr_policy_layout(ns, na, prec, off)
            assert size > 0 and all(0 <= o < size for o in off), (ns, na, prec, list(off), size)
    refused(lib.rr_policy_layout(10, 3, 0, None), "rr_policy_layout")
    refused(lib.rr_policy_layout(14, 3, 9, None), "rr_policy_layout")
    refused(lib.rr_policy_pack(14, 3, 0, None, fake, None), "rr_policy_pack")
    refused(lib.rr_policy_pack(14, 3, 0, _ptrs(13, null_at=12), fake, None), "rr_policy_pack")
    refused(lib.rr_policy_act(fake, 14, 3, 0, 0, 0, fake, 1, fake, 0, fake, fake, fake, fake, None, None, None, None,
                              0.99, None, None, None, None), "rr_policy_act")
    refused(lib.rr_policy_act(V(0x10004), 14, 3, 0, 64, 0, fake, 1, fake, 0, fake, fake, fake, fake, None, None, None,
                              None, 0.99, None, None, None, None), "rr_policy_act")  # params not 16-B aligned
    refused(lib.rr_policy_bootstrap(fake, 14, 3, 0, 64, None, None, None, 0.99, None, None, None, None),
            "rr_policy_bootstrap")  # nothing to do
    refused(lib.rr_policy_bootstrap(fake, 14, 3, 0, 64, fake, None, None, 0.99, None, None, None, None),
            "rr_policy_bootstrap")  # term_obs without truncated / reward / reward_out
    # PPO learner: workspace sizes (host only) and refusals, the 13-tensor lists read to the end
    ws = ctypes.c_int64()
    assert lib.rr_ppo_workspace_size(14, 3, 65536, ctypes.byref(ws)) == 0 and ws.value > 0
    small = ws.value
    assert lib.rr_ppo_workspace_size(14, 3, 2, ctypes.byref(ws)) == 0 and 0 < ws.value <= small
    refused(lib.rr_ppo_workspace_size(14, 3, 1, ctypes.byref(ws)), "rr_ppo_workspace_size")
    refused(lib.rr_ppo_workspace_size(5, 3, 64, ctypes.byref(ws)), "rr_ppo_workspace_size")
    args = [fake] * 6  # obs, actions, old_log_prob, advantages, returns, idx
    refused(lib.rr_ppo_grad(14, 3, None, _ptrs(13), *args, 64, ctypes.c_float(0.2), ctypes.c_float(0.01),
                            ctypes.c_float(0.5), None, fake, 1 << 30, None), "rr_ppo_grad")
    refused(lib.rr_ppo_grad(14, 3, _ptrs(13), _ptrs(13), *args, 64, ctypes.c_float(0.2), ctypes.c_float(0.01),
                            ctypes.c_float(0.5), None, fake, 16, None), "rr_ppo_grad")  # workspace too small
    refused(lib.rr_ppo_grad(14, 3, _ptrs(13), _ptrs(13), *args, 64, ctypes.c_float(0.2), ctypes.c_float(0.01),
                            ctypes.c_float(0.5), None, V(0x10008), 1 << 30, None), "rr_ppo_grad")  # misaligned
    refused(lib.rr_ppo_grad(14, 3, _ptrs(13), _ptrs(13), *args, 64, ctypes.c_float(-1.0), ctypes.c_float(0.01),
                            ctypes.c_float(0.5), None, fake, 1 << 30, None), "rr_ppo_grad")  # clip_range < 0
    refused(lib.rr_ppo_grad(14, 3, _ptrs(13), _ptrs(13, null_at=12), *args, 64, ctypes.c_float(0.2),
                            ctypes.c_float(0.01), ctypes.c_float(0.5), None, fake, 1 << 30, None), "rr_ppo_grad")
    assert lib.rr_clip_adam_workspace_size(42000, ctypes.byref(ws)) == 0 and ws.value >= 4
    refused(lib.rr_clip_adam_workspace_size(0, ctypes.byref(ws)), "rr_clip_adam_workspace_size")
    numel = (ctypes.c_int64 * 13)(*([64 * 14] * 13))
    lr = V(0x20000)

    def adam(n, params, numel_, ws_bytes):
        return lib.rr_clip_adam(n, params, _ptrs(13), _ptrs(13), _ptrs(13), _ptrs(13), numel_, ctypes.c_float(0.5),
                                lr, ctypes.c_double(0.9), ctypes.c_double(0.999), ctypes.c_float(1e-5), fake,
                                ws_bytes, None)

    refused(adam(0, _ptrs(13), numel, 1 << 20), "rr_clip_adam")
    refused(adam(17, _ptrs(13), numel, 1 << 20), "rr_clip_adam")
    refused(adam(13, _ptrs(13, null_at=12), numel, 1 << 20), "rr_clip_adam")
    numel[12] = 0
    refused(adam(13, _ptrs(13), numel, 1 << 20), "rr_clip_adam")  # empty tensor
    numel[12] = 64
    refused(adam(13, _ptrs(13), numel, 8), "rr_clip_adam")  # workspace too small
    # ABI 12: the chained minibatch step (rr_ppo_grad + rr_clip_adam in one call)
    assert lib.rr_ppo_update_workspace_size(14, 3, 65536, ctypes.byref(ws)) == 0 and ws.value > small
    refused(lib.rr_ppo_update_workspace_size(14, 3, 1, ctypes.byref(ws)), "rr_ppo_update_workspace_size")
    refused(lib.rr_ppo_update_workspace_size(9, 3, 64, ctypes.byref(ws)), "rr_ppo_update_workspace_size")

    def update(params=None, state_null=None, batch=64, nxt=None, next_batch=0, clip=0.2, flags=0, wsp=fake,
               ws_bytes=1 << 30):
        lists = [_ptrs(13, null_at=12) if state_null == k else _ptrs(13) for k in range(4)]
        return lib.rr_ppo_update(14, 3, _ptrs(13) if params is None else params, *lists, *args, batch, nxt,
                                 next_batch, ctypes.c_float(clip), ctypes.c_float(0.01), ctypes.c_float(0.5),
                                 ctypes.c_float(0.5), lr, ctypes.c_double(0.9), ctypes.c_double(0.999),
                                 ctypes.c_float(1e-5), None, flags, wsp, ws_bytes, None)

    refused(update(params=_ptrs(13, null_at=3)), "rr_ppo_update")
    for k in range(4):  # grads, exp_avg, exp_avg_sq, step
        refused(update(state_null=k), "rr_ppo_update")
    refused(update(batch=1), "rr_ppo_update")
    refused(update(ws_bytes=16), "rr_ppo_update")  # workspace too small
    refused(update(wsp=V(0x10008)), "rr_ppo_update")  # misaligned
    refused(update(clip=-1.0), "rr_ppo_update")
    refused(update(flags=0x2), "rr_ppo_update")  # unknown flag
    refused(update(nxt=fake, next_batch=1), "rr_ppo_update")
    refused(update(nxt=fake, next_batch=65), "rr_ppo_update")  # longer than this minibatch
    # rollouts / GAE (kept from ABI 3-7)
    refused(lib.rr_gae(16, 0, fake, fake, fake, fake, fake, ctypes.c_float(0.99), ctypes.c_float(0.95), fake, fake,
                       None), "rr_gae")
