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
