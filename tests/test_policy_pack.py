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
    g = lambda t: t.detach().numpy()  # noqa: E731
    for tw, net in ((o["PI"], pol.pi_net), (o["VF"], pol.vf_net)):
        w1, b1, w2, b2 = g(net[0].weight), g(net[0].bias), g(net[2].weight), g(net[2].bias)
        for m in range(2):
            for s in range(kp1):
                for lane in range(64):
                    k = 2 * s + (lane >> 5)
                    ref = w1[32 * m + (lane & 31), k] if k < ns else 0.0
                    assert buf[tw + o["L1A"] + (m * kp1 + s) * 64 + lane] == ref
            for half in range(2):
                for reg in range(16):
                    assert buf[tw + o["B1"] + (m * 2 + half) * 16 + reg] == b1[32 * m + _row(reg, half)]
                    assert buf[tw + o["B2"] + (m * 2 + half) * 16 + reg] == b2[32 * m + _row(reg, half)]
            for t in range(2):
                for gg in range(4):
                    for lane in range(64):
                        for r in range(4):
                            ref = w2[32 * m + (lane & 31), 32 * t + _row(4 * gg + r, lane >> 5)]
                            assert buf[tw + o["L2A"] + (((m * 2 + t) * 4 + gg) * 64 + lane) * 4 + r] == ref
    wa, wv = g(pol.action_net.weight), g(pol.value_net.weight)
    for a in range(na):
        for m in range(2):
            for half in range(2):
                for reg in range(16):
                    assert buf[o["HA"] + a * 64 + (m * 2 + half) * 16 + reg] == wa[a, 32 * m + _row(reg, half)]
    for m in range(2):
        for half in range(2):
            for reg in range(16):
                assert buf[o["HV"] + (m * 2 + half) * 16 + reg] == wv[0, 32 * m + _row(reg, half)]
    assert np.array_equal(buf[o["HB"]:o["HB"] + na], g(pol.action_net.bias))
    assert buf[o["VB"]] == g(pol.value_net.bias)[0]
    assert np.array_equal(buf[o["LS"]:o["LS"] + na], g(pol.log_std))
    assert pk.size == o["LS"] + 4


def test_layout_rejects_unsupported_dims():
    from rl_rocket_amd import _lib

    assert _lib.load(require_torch=False).rr_policy_layout(10, 3, None) == _lib.RR_EINVAL
