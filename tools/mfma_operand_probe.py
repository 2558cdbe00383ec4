"""MFMA operand-register probe: cycles per v_mfma_f32_32x32x2_f32 in a 64-MFMA burst (one wave per
SIMD, four accumulators in turn) by which VGPRs supply the A and B operands.

    python tools/mfma_operand_probe.py gen        # writes tools/mfma_operand_probe.hip
    hipcc --offload-arch=gfx950 -O2 -o tools/ab/mfma_operand_probe tools/mfma_operand_probe.hip
    tools/ab/mfma_operand_probe                   # on the GPU: one line per variant

Why: in the rollout collect the layer-2 MFMAs ran at ~130 cycles each, the layer-1 MFMAs at ~67
(tools/collect_stamps.py), and a layer-2 variant whose B operand was one fixed register (or an
inline constant) at 64. Each variant here is a hand-written burst (inline asm, explicit
registers), so the compiler's choices are out of the picture.
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ACC = ["v[0:15]", "v[16:31]", "v[32:47]", "v[48:63]"]


def burst(pairs, filler=None, k=0):
    """64 MFMAs; MFMA i accumulates into ACC[i % 4] with A = v pairs[i][0], B = v pairs[i][1]; after
    each, k independent filler instructions (filler(j) -> text, registers v100..v199)"""
    out = []
    j = 0
    for i, (a, b) in enumerate(pairs):
        out.append("v_mfma_f32_32x32x2_f32 %s, v%d, v%d, %s" % (ACC[i % 4], a, b, ACC[i % 4]))
        for _ in range(k):
            out.append(filler(j))
            j += 1
    return out


FILLERS = {
    "exp": lambda j: "v_exp_f32 v%d, v%d" % (160 + j % 40, 234 + j % 16),
    "rcp": lambda j: "v_rcp_f32 v%d, v%d" % (160 + j % 40, 234 + j % 16),
    "fma": lambda j: "v_fma_f32 v%d, v%d, v%d, v%d" % (160 + j % 40, 234 + j % 16, 235 + j % 14, 236 + j % 12),
    "pkfma": lambda j: "v_pk_fma_f32 v[%d:%d], v[%d:%d], v[%d:%d], v[%d:%d]" % (
        160 + 2 * (j % 20), 161 + 2 * (j % 20), 234 + 2 * (j % 7), 235 + 2 * (j % 7), 246, 247, 248, 249),
    "pkadd": lambda j: "v_pk_add_f32 v[%d:%d], v[%d:%d], v[%d:%d]" % (
        160 + 2 * (j % 20), 161 + 2 * (j % 20), 234 + 2 * (j % 7), 235 + 2 * (j % 7), 248, 249),
}
MIXES = [("exp", 1), ("exp", 2), ("exp", 4), ("exp", 8), ("rcp", 4), ("fma", 4), ("fma", 8), ("fma", 16),
         ("pkfma", 4), ("pkfma", 8), ("pkadd", 8)]


def variants():
    v = {}
    v["fixedA_fixedB"] = [(64, 65)] * 64
    v["fixedA_B16low"] = [(64, 65 + (i % 16)) for i in range(64)]
    v["fixedA_B16high"] = [(64, 200 + (i % 16)) for i in range(64)]
    v["fixedA_B64distinct"] = [(64, 120 + i) for i in range(64)]
    v["A4_B16low"] = [(64 + (i % 4), 70 + (i % 16)) for i in range(64)]
    # the compiled layer-2 pattern: per k step r (A0,B0),(A1,B0),(A1,B1),(A0,B1); A from two float4
    # groups, B the k-th register of two layer-1 tiles
    l2 = []
    for g in range(4):
        for r in range(4):
            a0, a1 = 84 + r, 150 + r
            b0, b1 = 90 + 4 * g + r, 218 + 4 * g + r
            l2 += [(a0, b0), (a1, b0), (a1, b1), (a0, b1)]
    v["l2_pattern"] = l2
    # same pattern with B registers in the same bank as their A (index mod 4 equal) / different
    l2b = []
    for g in range(4):
        for r in range(4):
            a0, a1 = 84 + r, 150 + r
            b0, b1 = 92 + 4 * g + ((r + 1) % 4), 216 + 4 * g + ((r + 1) % 4)
            l2b += [(a0, b0), (a1, b0), (a1, b1), (a0, b1)]
    v["l2_pattern_bankshift"] = l2b
    # the compiled layer-1 pattern: pairs share A
    l1 = []
    for s in range(8):
        for m in range(2):
            a = 86 + m
            l1 += [(a, 78 + s), (a, 100 + s)]
    v["l1_pattern"] = (l1 * 2)[:64]
    # B written by the previous burst's MFMA (an accumulator register of another tile)
    v["B_from_acc_regs"] = [(64, 16 * ((i + 2) % 4) + (i % 16)) for i in range(64)]
    return v


DATA = {  # operand values loaded into v0..v249 before the burst (numpy expression of rng, shape [250, 64])
    "d_affine": None,  # the original init (c2 + c1 * lane)
    "d_unit": "rng.uniform(-1, 1, (250, 64))",
    "d_sigmoid": "1 / (1 + 2.0 ** rng.uniform(-4, 4, (250, 64)))",
    "d_wide_exp": "rng.choice([-1, 1], (250, 64)) * 2.0 ** rng.uniform(-30, 30, (250, 64))",
    "d_denormal": "np.where(rng.uniform(0, 1, (250, 64)) < 0.1, 1e-40, rng.uniform(-1, 1, (250, 64)))",
    "d_zero_half": "np.where(rng.uniform(0, 1, (250, 64)) < 0.5, 0.0, rng.uniform(-1, 1, (250, 64)))",
    "d_bf16": "(rng.uniform(-1, 1, (250, 64)).astype(np.float32).view(np.uint32) & 0xFFFF0000).view(np.float32)",
    "d_big": "rng.uniform(-1, 1, (250, 64)) * 1e20",
}


def gen_data(path):
    """the operand images of the DATA variants, [variant][250][64] float32, for the probe binary"""
    import numpy as np
    rng = np.random.default_rng(11)
    arrs = []
    for name, expr in DATA.items():
        if expr is None:
            arrs.append(np.zeros((250, 64), np.float32))
        else:
            arrs.append(np.asarray(eval(expr), dtype=np.float64).astype(np.float32).reshape(250, 64))
    np.stack(arrs).astype(np.float32).tofile(path)


def gen():
    rnd = random.Random(7)
    out = ['// generated by tools/mfma_operand_probe.py (see its docstring); MFMA issue-rate probe, not product code',
           '#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <algorithm>', '']
    init = ["v_mbcnt_lo_u32_b32 v255, -1, 0", "v_mbcnt_hi_u32_b32 v255, -1, v255", "v_cvt_f32_u32 v255, v255"]
    for k in range(0, 250):
        c1, c2 = rnd.uniform(0.001, 0.02), rnd.uniform(-1.0, 1.0)
        init.append("v_fma_f32 v%d, v255, %r, %r" % (k, c1, c2) if False else
                    "v_mov_b32 v%d, %s" % (k, _hexf(c2)))
        init.append("v_fmac_f32 v%d, %s, v255" % (k, _hexf(c1)))
    clob = ", ".join('"v%d"' % k for k in range(256))
    names = []
    for name, pairs in variants().items():
        names.append(name)
        body = init + ["s_nop 7", "s_nop 7", "s_waitcnt lgkmcnt(0)", "s_memtime %0", "s_waitcnt lgkmcnt(0)"]
        body += burst(pairs)
        body += ["s_nop 7", "s_nop 7", "s_nop 7", "v_mov_b32 v250, v0", "v_mov_b32 v250, v16", "v_mov_b32 v250, v32",
                 "v_mov_b32 v250, v48", "s_memtime %1", "s_waitcnt lgkmcnt(0)"]
        asm = "\\n\\t".join(body)
        out.append("__global__ __launch_bounds__(256) void k_%s(unsigned long long* out)" % name)
        out.append("{")
        out.append("    unsigned long long t0, t1;")
        out.append('    asm volatile("%s" : "=&s"(t0), "=&s"(t1) : : %s, "memory");' % (asm, clob))
        out.append("    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;")
        out.append("}")
        out.append("")
    for fname, k in MIXES:
        name = "mix_%s%d" % (fname, k)
        names.append(name)
        body = init + ["s_nop 7", "s_nop 7", "s_waitcnt lgkmcnt(0)", "s_memtime %0", "s_waitcnt lgkmcnt(0)"]
        body += burst(variants()["l2_pattern"], FILLERS[fname], k)
        body += ["s_nop 7", "s_nop 7", "s_nop 7", "v_mov_b32 v250, v0", "v_mov_b32 v250, v16", "v_mov_b32 v250, v32",
                 "v_mov_b32 v250, v48", "s_memtime %1", "s_waitcnt lgkmcnt(0)"]
        asm = "\\n\\t".join(body)
        out.append("__global__ __launch_bounds__(256) void k_%s(unsigned long long* out)" % name)
        out.append("{")
        out.append("    unsigned long long t0, t1;")
        out.append('    asm volatile("%s" : "=&s"(t0), "=&s"(t1) : : %s, "memory");' % (asm, clob))
        out.append("    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;")
        out.append("}")
        out.append("")
    # l2 pattern on loaded operand values (DATA); v254 = lane * 4, v253 = block base
    ld = ["v_mbcnt_lo_u32_b32 v254, -1, 0", "v_mbcnt_hi_u32_b32 v254, -1, v254", "v_lshlrev_b32 v254, 2, v254"]
    for blk in range(0, 250, 15):
        ld.append("v_add_u32 v253, %d, v254" % (blk * 256))
        for j in range(blk, min(blk + 15, 250)):
            ld.append("global_load_dword v%d, v253, %%2 offset:%d" % (j, (j - blk) * 256))
    ld.append("s_waitcnt vmcnt(0)")
    pairs = variants()["l2_pattern"]
    for dname in DATA:
        if DATA[dname] is None:
            continue
        name = "l2_" + dname
        names.append(name)
        body = ld + ["s_nop 7", "s_waitcnt lgkmcnt(0)", "s_memtime %0", "s_waitcnt lgkmcnt(0)"] + burst(pairs)
        body += ["s_nop 7", "s_nop 7", "s_nop 7", "v_mov_b32 v250, v0", "v_mov_b32 v250, v16", "v_mov_b32 v250, v32",
                 "v_mov_b32 v250, v48", "s_memtime %1", "s_waitcnt lgkmcnt(0)"]
        asm = "\\n\\t".join(body)
        out.append("__global__ __launch_bounds__(256) void k_%s(unsigned long long* out, const float* vals)" % name)
        out.append("{")
        out.append("    unsigned long long t0, t1;")
        out.append('    asm volatile("%s" : "=&s"(t0), "=&s"(t1) : "s"(vals) : %s, "memory");' % (asm, clob))
        out.append("    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;")
        out.append("}")
        out.append("")
    out.append("int main()")
    out.append("{")
    out.append("    const int W = 1024;")
    out.append("    unsigned long long* d;")
    out.append("    if (hipMalloc(&d, W * 8) != hipSuccess) return 1;")
    out.append("    std::vector<unsigned long long> h(W);")
    out.append("    const int NV = %d;" % len(DATA))
    out.append("    std::vector<float> hv((size_t)NV * 250 * 64);")
    out.append('    FILE* f = fopen("tools/ab/mfma_operand_probe.dat", "rb");')
    out.append("    if (!f || fread(hv.data(), 4, hv.size(), f) != hv.size()) return 3;")
    out.append("    fclose(f);")
    out.append("    float* dv;")
    out.append("    if (hipMalloc(&dv, hv.size() * 4) != hipSuccess) return 1;")
    out.append("    hipMemcpy(dv, hv.data(), hv.size() * 4, hipMemcpyHostToDevice);")
    dnames = list(DATA)
    for name in names:
        arg = ""
        if name.startswith("l2_d_"):
            arg = ", dv + (size_t)%d * 250 * 64" % dnames.index(name[3:])
        out.append("    for (int rep = 0; rep < 3; ++rep) {")
        out.append("        hipLaunchKernelGGL(k_%s, dim3(256), dim3(256), 0, 0, d%s);" % (name, arg))
        out.append("        if (hipDeviceSynchronize() != hipSuccess) return 2;")
        out.append("    }")
        out.append("    hipMemcpy(h.data(), d, W * 8, hipMemcpyDeviceToHost);")
        out.append("    std::sort(h.begin(), h.end());")
        out.append('    printf("%%-24s median %%7.1f  p10 %%7.1f  p90 %%7.1f cycles per MFMA\\n", "%s", h[W / 2] / 64.0, '
                   'h[W / 10] / 64.0, h[9 * W / 10] / 64.0);' % name)
    out.append("    hipFree(d);")
    out.append("    return 0;")
    out.append("}")
    with open(os.path.join(HERE, "mfma_operand_probe.hip"), "w") as f:
        f.write("\n".join(out) + "\n")


def _hexf(x):
    import struct
    return "0x%08x" % struct.unpack("<I", struct.pack("<f", x))[0]


if __name__ == "__main__":
    if sys.argv[1:] == ["gen"]:
        gen()
        gen_data(os.path.join(HERE, "ab", "mfma_operand_probe.dat"))
