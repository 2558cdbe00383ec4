"""gym 0.21 seeding / Box restatement used by the single-env shims' host-side reset.

Pinned against the reset ICs the reference produced in the survey container
(tests/golden, G8). NOTE: those were generated with the gym-0.21 restatement in
tests/golden/_shim (gym is absent from the image), so this pins the two restatements
to each other and to the reference's own reset()/float32 quaternion normalisation —
not to a real gym install."""
import numpy as np

from rl_rocket_amd import gym_compat as G
from rl_rocket_amd import params as P


def _resets(cfg, k, normalize_q):
    box = G.Box(low=cfg.ic_low, high=cfg.ic_high)
    box.seed(cfg.kwargs["seed"])
    out = []
    for _ in range(k):
        ic = box.sample()
        if normalize_q:
            ic[6:10] = ic[6:10] / np.linalg.norm(ic[6:10])
        out.append(ic)
    return np.array(out)


def test_6dof_reset_stream(golden6):
    r = _resets(P.config_6dof(**P.ENV_CONFIG_6DOF), 32, True)
    assert np.array_equal(r, golden6["resets_seed42"])
    r = _resets(P.config_6dof(), 8, True)
    assert np.array_equal(r, golden6["resets_default_seed42"])


def test_3dof_reset_stream(golden3):
    r = _resets(P.config_3dof(), 32, False)
    assert np.array_equal(r, golden3["resets_seed42"])


def test_box_contains_semantics():
    b = G.Box(low=np.float32([-30, -135, -135]), high=np.float32([540, 135, 135]))
    assert b.contains(np.float32([540, 135, -135]))          # inclusive
    assert not b.contains(np.float32([540.0001, 0, 0]))
    assert not b.contains(np.float32([np.nan, 0, 0]))          # NaN -> outside -> done
    assert not b.contains(np.float64([0, 0, 0]))              # can_cast(float64 -> float32) is False
