"""CPU: the fragment-ordered parameter layout of the fused rollout policy kernel
(rl_rocket_amd/csrc/rocket_policy.inc), PyTorch packer vs an independent loop restatement
of the documented layout. rr_policy_layout is host-only (no GPU needed)."""
import numpy as np
import pytest


def _row(reg, half):
    return (reg & 3) + 8 * (reg >> 2) + 4 * half


@pytest.mark.parametrize("ns,na", [(14, 3), (7, 2)])
def test_pack_reference_matches_layout(ns, na):
    import torch
    from rl_rocket_amd.rollout import MlpActorCritic, PolicyPack

    torch.manual_seed(1)
    pol = MlpActorCritic(ns, na)
    with torch.no_grad():
        for p in pol.parameters():
            p.add_(torch.randn_like(p))
    pk = PolicyPack(pol, ns, na, torch.device("cpu"))
    buf = pk.pack_reference().numpy()
    o = pk.off
    kp1 = (ns + 1) // 2
    g = lambda t: t.detach().numpy().astype(np.float64)  # noqa: E731
    # the folded fp32 tanh (rocket_policy.inc kPolFoldTanh; tanh(x) = 1 - 2 / (1 + 2^(c x))): c = 2 log2 e
    # on layer 1, -2c on W2 and c (b2 + row sums of W2) on b2, -2 on the head weights and + row sums on
    # their biases; fp64, one rounding to fp32
    c = 2.0 * np.log2(np.e)
    f32 = np.float32

    def rowsum(w):  # column by column, as the pack kernel
        acc = np.zeros(w.shape[0])
        for q in range(w.shape[1]):
            acc = acc + w[:, q]
        return acc

    for tw, net in ((o["PI"], pol.pi_net), (o["VF"], pol.vf_net)):
        w1, b1, w2, b2 = g(net[0].weight), g(net[0].bias), g(net[2].weight), g(net[2].bias)
        b2f = b2 + rowsum(w2)
        for m in range(2):
            for s in range(kp1):
                for lane in range(64):
                    k = 2 * s + (lane >> 5)
                    ref = f32(c * w1[32 * m + (lane & 31), k]) if k < ns else 0.0
                    assert buf[tw + o["L1A"] + (m * kp1 + s) * 64 + lane] == ref
            for half in range(2):
                for reg in range(16):
                    assert buf[tw + o["B1"] + (m * 2 + half) * 16 + reg] == f32(c * b1[32 * m + _row(reg, half)])
                    assert buf[tw + o["B2"] + (m * 2 + half) * 16 + reg] == f32(c * b2f[32 * m + _row(reg, half)])
            for t in range(2):
                for gg in range(4):
                    for lane in range(64):
                        for r in range(4):
                            ref = f32(-2.0 * c * w2[32 * m + (lane & 31), 32 * t + _row(4 * gg + r, lane >> 5)])
                            assert buf[tw + o["L2A"] + (((m * 2 + t) * 4 + gg) * 64 + lane) * 4 + r] == ref
    wa, wv = g(pol.action_net.weight), g(pol.value_net.weight)
    for a in range(na):
        for m in range(2):
            for half in range(2):
                for reg in range(16):
                    assert buf[o["HA"] + a * 64 + (m * 2 + half) * 16 + reg] == -2.0 * wa[a, 32 * m + _row(reg, half)]
    for m in range(2):
        for half in range(2):
            for reg in range(16):
                assert buf[o["HV"] + (m * 2 + half) * 16 + reg] == -2.0 * wv[0, 32 * m + _row(reg, half)]
    assert np.array_equal(buf[o["HB"]:o["HB"] + na], (g(pol.action_net.bias) + rowsum(wa)).astype(f32))
    assert buf[o["VB"]] == f32(g(pol.value_net.bias)[0] + rowsum(wv)[0])
    assert np.array_equal(buf[o["LS"]:o["LS"] + na], g(pol.log_std))
    assert pk.size == o["LS"] + 4


@pytest.mark.parametrize("ns,na", [(14, 3), (7, 2)])
def test_pack_reference_bf16_matches_layout(ns, na):
    """bf16 tower sections: 8 RNE bf16 per lane and k step, W2 in the permuted k order of
    an accumulator tile used as the next MFMA's B operand (rocket_policy.inc)."""
    import torch
    from rl_rocket_amd.rollout import MlpActorCritic, PolicyPack

    torch.manual_seed(2)
    pol = MlpActorCritic(ns, na)
    with torch.no_grad():
        for p in pol.parameters():
            p.add_(torch.randn_like(p))
    pk = PolicyPack(pol, ns, na, torch.device("cpu"), precision="bf16")
    bits = pk.pack_reference().view(torch.int32).numpy().view(np.uint16)  # 2 bf16 per float, low half first
    fl = pk.buf.numpy()
    o = pk.off
    kp1 = (ns + 15) // 16

    def bf(x):  # RNE bf16 bits of an fp32 value
        return int(torch.tensor([float(x)], dtype=torch.float32).to(torch.bfloat16).view(torch.int16).item()) & 0xFFFF

    g = lambda t: t.detach().numpy()  # noqa: E731
    for tw, net in ((o["PI"], pol.pi_net), (o["VF"], pol.vf_net)):
        w1, b1, w2, b2 = g(net[0].weight), g(net[0].bias), g(net[2].weight), g(net[2].bias)
        for m in range(2):
            for s in range(kp1):
                for lane in range(64):
                    for j in range(8):
                        k = 16 * s + 8 * (lane >> 5) + j
                        ref = bf(w1[32 * m + (lane & 31), k]) if k < ns else 0
                        assert bits[2 * (tw + o["L1A"]) + ((m * kp1 + s) * 64 + lane) * 8 + j] == ref
            for half in range(2):
                for reg in range(16):
                    assert fl[tw + o["B1"] + (m * 2 + half) * 16 + reg] == b1[32 * m + _row(reg, half)]
                    assert fl[tw + o["B2"] + (m * 2 + half) * 16 + reg] == b2[32 * m + _row(reg, half)]
            for t in range(2):
                for s in range(2):
                    for lane in range(64):
                        for j in range(8):
                            col = 32 * t + 16 * s + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3)
                            # the same k as D-tile register 8s + j of lane half h
                            assert col == 32 * t + _row(8 * s + j, lane >> 5)
                            ref = bf(w2[32 * m + (lane & 31), col])
                            assert bits[2 * (tw + o["L2A"]) + (((m * 2 + t) * 2 + s) * 64 + lane) * 8 + j] == ref
    assert o["B1"] == 2 * kp1 * 64 * 4 and o["B2"] - o["L2A"] == 2048
    assert pk.size == o["LS"] + 4


def test_layout_rejects_unsupported_dims():
    from rl_rocket_amd import _lib

    lib = _lib.load(require_torch=False)
    assert lib.rr_policy_layout(10, 3, _lib.RR_POLICY_FP32, None) == _lib.RR_EINVAL
    assert lib.rr_policy_layout(14, 3, 3, None) == _lib.RR_EINVAL  # unknown precision
    assert lib.rr_policy_layout(14, 3, _lib.RR_POLICY_BF16, None) < lib.rr_policy_layout(14, 3, 0, None)


@pytest.mark.parametrize("ns,na", [(14, 3), (7, 2)])
def test_pack_reference_fp16x3_matches_layout(ns, na):
    """split-fp16 tower sections: [hi, lo] fp16 planes of 2^8 W in the bf16 fragment order;
    hi + lo reproduces 2^8 W to 2^-21 relative (22 significant bits), biases packed at the
    2^16 accumulator scale."""
    import torch
    from rl_rocket_amd.rollout import MlpActorCritic, PolicyPack

    torch.manual_seed(5)
    pol = MlpActorCritic(ns, na)
    with torch.no_grad():
        for prm in pol.parameters():
            prm.add_(0.3 * torch.randn_like(prm))
    pk = PolicyPack(pol, ns, na, torch.device("cpu"), precision="fp16x3")
    buf = pk.pack_reference()
    o, kp1 = pk.off, (ns + 15) // 16
    plane1, plane2 = 2 * kp1 * 64 * 4, 2048
    assert o["B1"] == 2 * plane1 and o["B2"] - o["L2A"] == 2 * plane2
    f16 = buf.view(torch.int32).numpy().view(np.float16).astype(np.float64)  # 2 halves per float, low first
    for tw, net in ((o["PI"], pol.pi_net), (o["VF"], pol.vf_net)):
        w1 = torch.nn.functional.pad(net[0].weight.detach(), (0, 16 * kp1 - ns)).double().numpy()
        w2 = net[2].weight.detach().double().numpy()
        hi1 = f16[2 * (tw + o["L1A"]): 2 * (tw + o["L1A"] + plane1)]
        lo1 = f16[2 * (tw + o["L1A"] + plane1): 2 * (tw + o["L1A"] + 2 * plane1)]
        hi2 = f16[2 * (tw + o["L2A"]): 2 * (tw + o["L2A"] + plane2)]
        lo2 = f16[2 * (tw + o["L2A"] + plane2): 2 * (tw + o["L2A"] + 2 * plane2)]
        ref1 = 256.0 * w1[pk.l1_i.numpy(), pk.l1_k.numpy()]
        ref2 = 256.0 * w2[pk.l2_i.numpy(), pk.l2_k.numpy()]
        for hi, lo, ref in ((hi1, lo1, ref1), (hi2, lo2, ref2)):
            err = np.abs(hi + lo - ref) / np.maximum(np.abs(ref), 1e-3)
            assert err.max() < 2.0 ** -20, err.max()
            assert np.all(np.abs(lo) <= np.abs(hi) * 2.0 ** -10 + 2.0 ** -24)
        b1 = buf[tw + o["B1"]: tw + o["B1"] + 64].numpy()
        assert np.array_equal(b1, (net[0].bias.detach()[pk.b_i] * 65536.0).numpy())
