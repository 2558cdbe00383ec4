"""my_environment.wrappers: ``RewardAnnealing`` (reference wrappers.py:68-86) restated over
the shims. The plotting / logging wrappers (EpisodeAnalyzer*, RecordVideoFigure,
GaudetStateObs, DiscreteActions3DOF: wandb, plotly, pygame) are out of scope and raise.

For vectorised training use ``rl_rocket_amd.RocketVecEnv(..., reward_annealing=True)``,
which computes the annealed reward inside the step kernel.
"""
from rl_rocket_amd.envs import Rocket6DOF
from rl_rocket_amd.gym_compat import HAVE_GYM

if HAVE_GYM:  # pragma: no cover
    import gym

    _Base = gym.Wrapper
else:
    class _Base:
        def __init__(self, env):
            self.env = env
            self.action_space = env.action_space
            self.observation_space = env.observation_space

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)
            return getattr(self.env, name)

        @property
        def unwrapped(self):
            return getattr(self.env, "unwrapped", self.env)

        def reset(self, **kw):
            return self.env.reset(**kw)

        def step(self, action):
            return self.env.step(action)


class RewardAnnealing(_Base):
    """reward = attitude_constraint + rew_goal - xi * (a_thrust + 1) (wrappers.py:72-86)."""

    def __init__(self, env, thrust_penalty: float = 0.01):
        super().__init__(env)
        self.xi = self.reward_coefficients.get("xi", thrust_penalty)

    def step(self, action):
        obs, _, done, info = self.env.step(action)
        old = info["rewards_dict"]
        rewards_dict = {k: old[k] for k in ("attitude_constraint", "rew_goal")}
        a_t = action[2] if isinstance(self.unwrapped, Rocket6DOF) else action[1]
        rewards_dict["thrust_penalty"] = -self.xi * (a_t + 1)
        info["rewards_dict"] = rewards_dict
        return obs, sum(rewards_dict.values()), done, info


def _out_of_scope(name):
    def _raise(*a, **k):
        raise NotImplementedError("%s (wandb / plotly / pygame visualisation) is out of scope of rl_rocket_amd" % name)
    return _raise


EpisodeAnalyzer = _out_of_scope("EpisodeAnalyzer")
EpisodeAnalyzer6DOF = _out_of_scope("EpisodeAnalyzer6DOF")
RecordVideoFigure = _out_of_scope("RecordVideoFigure")
GaudetStateObs = _out_of_scope("GaudetStateObs")
DiscreteActions3DOF = _out_of_scope("DiscreteActions3DOF")

__all__ = ["RewardAnnealing", "EpisodeAnalyzer", "EpisodeAnalyzer6DOF", "RecordVideoFigure", "GaudetStateObs",
           "DiscreteActions3DOF"]
