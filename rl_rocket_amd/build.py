"""Build ``librocket_hip.so`` in-tree with hipcc for gfx950 (MI355X).

    python -m rl_rocket_amd.build [--force] [--resource-usage]
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "rocket_hip.hip")
# the exact-mode kernels' translation unit (rocket_hip.hip again under RR_TU_EXACT), compiled with
# a register-pressure-first scheduler: with the fast kernels' setting the 6DOF exact kernel spilled
# 33 VGPRs to scratch at one wave per SIMD (r03e), with it none
SRC_EXACT = os.path.join(HERE, "csrc", "rocket_exact.hip")
EXACT_FLAGS = ["-mllvm", "-amdgpu-schedule-metric-bias=100"]
# the rollout collect and PPO learner kernels' translation unit (rocket_hip.hip under RR_TU_COLLECT),
# with the MFMA accumulators in VGPRs: no v_accvgpr_read per tanh input (5.5 % faster collect,
# round 4; the learner's minibatch 3 % faster, round 6)
SRC_COLLECT = os.path.join(HERE, "csrc", "rocket_collect.hip")
COLLECT_FLAGS = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
DEPS = [os.path.join(HERE, "csrc", f) for f in ("rocket_dopri5.inc", "rocket_policy.inc", "rocket_rollout.inc", "rocket_ppo.inc",
                                                 "rocket_exact.hip", "rocket_collect.hip",
                                                 "rocket_stamps.h")]
HEADER = os.path.join(ROOT, "include", "rocket_hip.h")
OUT = os.path.join(HERE, "librocket_hip.so")
# benchmark-only helper (not part of the product ABI): bench.py's event-timed direct-launch region
BENCH_SRC = os.path.join(ROOT, "tools", "bench_timed.hip")
BENCH_OUT = os.path.join(ROOT, "tools", "libbench_timed.so")
ARCH = os.environ.get("RR_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def command(resource_usage=False, out=OUT, defines=(), extra=(), src=SRC, compile_only=False, preload=4):
    # -fno-slp-vectorize: the SLP pass packs scalar f32 math into v_pk_* pairs and adds ~180
    # register moves to the step kernel (measured on the .s); the scalar stream is shorter.
    # -ffp-contract=on: a*b+c becomes an fma only inside one source expression. HIP's default
    # (fast) also fuses across statements in the backend, and what it fuses depends on the
    # basic-block layout around inlined code: the env step inlined into rr_rollout_step then
    # rounded differently from step_kernel (1 ulp in 0.2 % of envs). Expression-level
    # contraction makes every kernel that inlines the physics compute the same bits.
    # kernarg preload: the step kernel's leading pointer / word arguments arrive in user SGPRs
    cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-O3", "-fno-slp-vectorize", "-ffp-contract=on", "-std=c++17",
           "-fPIC", "-c" if compile_only else "-shared"] + \
        (["-mllvm", "-amdgpu-kernarg-preload-count=%d" % preload] if preload else []) + \
        ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc")] + list(extra) + \
        ["-D%s" % d for d in defines] + ["-o", out, src]
    if resource_usage:
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
    return cmd


def source_hash():
    """sha256 of everything that determines the kernels' code: the HIP sources, the C-ABI
    header and the compile command (tools/pmc_traffic.py stamps its output with it; bench.py
    only quotes a PMC traffic file measured on the same kernel code)."""
    import hashlib

    h = hashlib.sha256()
    for path in [SRC, HEADER] + DEPS:
        with open(path, "rb") as f:
            h.update(f.read())
    for cmd in commands():
        h.update(" ".join(cmd[1:]).replace(ROOT, "").encode())
    return h.hexdigest()[:16]


def commands(resource_usage=False, out=OUT, defines=(), extra=(), preload=4):
    """The four steps of the library build: the main, exact-mode and collect translation units
    compiled to objects (the latter two with EXACT_FLAGS / COLLECT_FLAGS), then linked into `out`."""
    o_main, o_exact, o_coll = out + ".main.o", out + ".exact.o", out + ".collect.o"
    c1 = command(resource_usage, o_main, defines, extra, SRC, compile_only=True, preload=preload)
    c2 = command(resource_usage, o_exact, defines, list(extra) + EXACT_FLAGS, SRC_EXACT, compile_only=True,
                 preload=preload)
    c3 = command(resource_usage, o_coll, defines, list(extra) + COLLECT_FLAGS, SRC_COLLECT, compile_only=True,
                 preload=preload)
    c4 = [hipcc(), "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-o", out, o_main, o_exact, o_coll]
    return [c1, c2, c3, c4]


def build_lib(out=OUT, defines=(), extra=(), resource_usage=False, verbose=True, preload=4):
    """Compile the three translation units (in parallel) and link `out`."""
    cmds = commands(resource_usage, out, defines, extra, preload=preload)
    if verbose:
        for c in cmds:
            print("[rl_rocket_amd.build]", " ".join(c), flush=True)
    procs = [subprocess.Popen(c, cwd=ROOT) for c in cmds[:-1]]
    rcs = [p.wait() for p in procs]
    for c, rc in zip(cmds, rcs):
        if rc:
            raise subprocess.CalledProcessError(rc, c)
    subprocess.check_call(cmds[-1], cwd=ROOT)
    for c in cmds[:-1]:
        os.remove(c[c.index("-o") + 1])
    return out


def _llvm(tool):
    for d in (os.environ.get("ROCM_PATH", "/opt/rocm") + "/lib/llvm/bin", "/opt/rocm/llvm/bin"):
        if os.path.exists(os.path.join(d, tool)):
            return os.path.join(d, tool)
    found = shutil.which(tool)
    if not found:
        raise RuntimeError("%s not found" % tool)
    return found


def _elf_symbols(blob):
    """(name, bytes) of the FUNC symbols and kernel descriptors (OBJECT *.kd) of an ELF64 blob."""
    import struct

    shoff, = struct.unpack_from("<Q", blob, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", blob, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", blob, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for sec in secs:
        if sec[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[sec[6]]
        for k in range(sec[5] // 24):
            name_off, info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", blob, sec[4] + 24 * k)
            if size == 0 or shndx == 0 or shndx >= len(secs) or (info & 0xF) not in (1, 2):  # OBJECT / FUNC
                continue
            so = strtab[4] + name_off
            name = blob[so:blob.index(b"\0", so)].decode()
            tsec = secs[shndx]
            start = tsec[4] + (value - tsec[3])
            out[name] = blob[start:start + size]
    return out


def kernel_isa_hashes(lib=OUT):
    """{demangled kernel name: sha256[:16] of its gfx950 machine code + kernel descriptor} of
    a built library: the identity of the code a profile measured, independent of unrelated
    edits elsewhere in the translation unit (bench.py quotes committed PMC / rocprofv3 figures
    only for the same ISA). Uses llvm-objcopy, clang-offload-bundler (ROCm) and c++filt."""
    import hashlib
    import tempfile

    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    syms = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.check_call([_llvm("llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, lib, os.path.join(d, "x")])
        with open(fat, "rb") as f:
            blob = f.read()
        starts, k = [], blob.find(magic)  # one bundle per translation unit
        while k >= 0:
            starts.append(k)
            k = blob.find(magic, k + len(magic))
        for n, k0 in enumerate(starts):
            k1 = starts[n + 1] if n + 1 < len(starts) else len(blob)
            part, co = os.path.join(d, "b%d.bin" % n), os.path.join(d, "b%d.co" % n)
            with open(part, "wb") as f:
                f.write(blob[k0:k1])
            subprocess.check_call([_llvm("clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + part,
                                   "--targets=hipv4-amdgcn-amd-amdhsa--%s" % ARCH, "--output=" + co])
            with open(co, "rb") as f:
                syms.update(_elf_symbols(f.read()))
    funcs = sorted(n for n in syms if not n.endswith(".kd"))
    names = subprocess.run(["c++filt"], input="\n".join(funcs), capture_output=True, text=True,
                           check=True).stdout.splitlines()
    out = {}
    for mangled, name in zip(funcs, names):
        h = hashlib.sha256(syms[mangled])
        kd = bytearray(syms.get(mangled + ".kd", b""))
        kd[16:24] = bytes(8)[:len(kd[16:24])]  # kernel_code_entry_byte_offset: where the code sits, not what it is
        h.update(bytes(kd))
        out[name] = h.hexdigest()[:16]
    return out


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in [SRC, HEADER, __file__] + DEPS)


def build(force=False, resource_usage=False, verbose=True):
    build_bench_helper(force=force, verbose=verbose)
    if not force and up_to_date():
        return OUT
    return build_lib(OUT, resource_usage=resource_usage, verbose=verbose)


def build_bench_helper(force=False, verbose=True):
    """tools/libbench_timed.so: the gate kernel + event-timed launch loop bench.py uses below
    K = 32 timed steps (it drives the library through its public rr_step)."""
    if not force and os.path.exists(BENCH_OUT) and os.path.getmtime(BENCH_OUT) >= os.path.getmtime(BENCH_SRC):
        return BENCH_OUT
    cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-o", BENCH_OUT, BENCH_SRC]
    if verbose:
        print("[rl_rocket_amd.build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=ROOT)
    return BENCH_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, resource_usage="--resource-usage" in sys.argv)
