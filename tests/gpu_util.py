"""Helpers shared by the GPU parity tests (tests only)."""
import numpy as np

# Parity tolerance of the north star: fp32 within 1e-5, measured floored-relative
# |a - b| / max(|b|, normalizer_c) on states/obs, |a - b| / max(|b|, 1)
# on reward terms.
TOL_STATE = 1e-5
TOL_REWARD = 1e-5


def floored_rel(a, b, floor):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), np.asarray(floor, np.float64))


def run_rows(model, rows, **env_kwargs):
    """Inject golden rows (state_in, ic, action) into a RocketBatch, step once,
    return host copies of every output."""
    import torch
    from rl_rocket_amd.batch import RocketBatch

    ns = 14 if model == 6 else 7
    n = len(rows["group"])
    b = RocketBatch(n, model=model, device="cuda:0", max_episode_steps=0, auto_reset=False, episode_stats=False,
                    compute_terms=True, **env_kwargs)
    ic = rows["ic"].astype(np.float32)
    v0 = np.sqrt((ic[:, 3:6 if model == 6 else 5].astype(np.float32) ** 2).sum(1, dtype=np.float32)).astype(np.float32)
    b.set_state(torch.from_numpy(rows["state_in"].astype(np.float32).T.copy()), v0=torch.from_numpy(v0))
    obs, rew, done, trunc = b.step(torch.from_numpy(rows["action"].astype(np.float32)))
    st, _, _ = b.get_state()
    torch.cuda.synchronize()
    out = dict(state_out=st.cpu().numpy().T.astype(np.float64), obs=obs.cpu().numpy(), reward=rew.cpu().numpy(),
               done=done.cpu().numpy().astype(bool), terms=b.terms.cpu().numpy().T)
    out["bounds_violation"] = out["terms"][:, -2] > 0.5
    out["event"] = out["terms"][:, -1] > 0.5
    out["terms"] = out["terms"][:, :-2]
    b.close()
    return out
