"""Drop-in ``masurvival.envs.masurvival_env.MaSurvival`` (demo.py:11,178-180).

Same surface as the reference env (masurvival_env.py:32-135, 241-929):
``MaSurvival(config)``, ``reset(seed=None, return_info=False, options=None)``,
``step(actions) -> (obs dict, rewards float32[A], done, {})``,
``observation_space`` / ``action_space``, ``n_agents`` / ``n_heals`` /
``n_boxes`` / ``has_teams``, ``flush_stats()``, ``close()``.  The step runs on
the GPU as a one-env VecMaSurvival (HIP kernels); observations come back as
the reference's dict of float32 numpy arrays.

Documented deviations: ``reset(seed=...)`` reseeds (the reference ignores
it, masurvival_env.py:58-66); an ``np_random`` assigned before ``reset`` is
injected into the device stream (the GPU then owns that stream);
``MaSurvival(config=None)`` can be constructed repeatedly (the reference
mutates its class-level defaults on the first construction);
``render()`` is out of scope (rendering is not on the hot path).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import numpy as np

from .. import spaces
from ..config import ResolvedConfig, onevsone_heals_config
from ..vec_env import VecMaSurvival

STAT_REWARD, STAT_KILLS, STAT_STEPS, STAT_HEALS, STAT_BOXES = 0, 8, 16, 17, 18


class MaSurvival:
    config = onevsone_heals_config
    metadata: Dict[str, Any] = {'render_modes': ['human', 'rgb_array'], 'render_fps': 30}

    def __init__(self, config: Optional[Dict[str, Dict[str, Any]]] = None, device=None):
        self.rc = ResolvedConfig(config)
        self.config = self.rc.config
        self._vec = VecMaSurvival(config, n_envs=1, device=device, auto_reset=False)
        self.np_random = np.random.default_rng()
        self._injected = None
        self.observation_space = self._vec.observation_space
        self.action_space = self._vec.action_space
        self.steps = 0
        self._stats_acc = None

    # reference properties (masurvival_env.py:245-279)
    @property
    def n_agents(self) -> int:
        return self.rc.n_agents

    @property
    def n_heals(self) -> int:
        return self.rc.n_heals

    @property
    def n_boxes(self) -> int:
        return self.rc.n_boxes

    @property
    def has_teams(self) -> bool:
        return self.rc.has_teams

    @property
    def box_ownership(self) -> bool:
        return self.rc.box_ownership

    def _inject_rng(self):
        if self._injected is self.np_random:
            return
        st = self.np_random.bit_generator.state
        s, inc = int(st['state']['state']), int(st['state']['inc'])
        m = (1 << 64) - 1
        arr = np.array([[s >> 64, s & m, inc >> 64, inc & m, int(st['has_uint32']), int(st['uinteger'])]],
                       dtype=np.uint64)
        self._vec.set_rng_states(arr)
        self._injected = self.np_random

    def _obs_dict(self, flat):
        host = flat[0].detach().cpu().numpy()
        x = {k: np.ascontiguousarray(v) for k, v in self._vec.split(host).items()}
        # fetch_observations' own check (masurvival_env.py:656)
        assert self.observation_space.contains(x), f'{x} not contained in the observation space {self.observation_space}'
        return x

    def reset(self, seed: Optional[int] = None, return_info: bool = False, options: Optional[Dict] = None):
        if seed is not None:
            self.np_random = np.random.default_rng(seed)
        self._inject_rng()
        obs = self._obs_dict(self._vec.reset())
        self.steps = 0
        return (obs, {}) if return_info else obs

    def step(self, actions) -> Tuple[Dict[str, np.ndarray], np.ndarray, bool, Dict]:
        actions = tuple(a for a in actions)
        assert self.action_space.contains(actions), f'Invalid action {actions}.'
        import torch
        a = torch.as_tensor(np.stack([np.asarray(x) for x in actions]).astype(np.int8)).reshape(1, self.n_agents, 6)
        obs, rew, done, _ = self._vec.step(a.to(self._vec.device))
        self.steps += 1
        return self._obs_dict(obs), rew[0].cpu().numpy().copy(), bool(done[0].item()), {}

    def flush_stats(self) -> Dict[str, float]:
        s = self._vec.flush_stats()[0].cpu().numpy()
        n_rewards = 2 if self.has_teams else self.n_agents
        stats = {f'reward{i}': float(s[STAT_REWARD + i]) for i in range(n_rewards)}
        for i in range(n_rewards):
            stats[f'kills{i}'] = int(s[STAT_KILLS + i])
        stats['steps'] = int(s[STAT_STEPS])
        stats['heals_used'] = int(s[STAT_HEALS])
        stats['boxes_placed'] = int(s[STAT_BOXES])
        return stats

    def render(self, mode: str = 'human'):
        """mode='rgb_array': a top-down uint8 [400, 400, 3] frame of the env
        from device state (masurvival.render); 'human' needs pygame, which
        this build does not have."""
        if mode != 'rgb_array':
            raise NotImplementedError("only render(mode='rgb_array') is available in the MI355X build")
        from masurvival.render import render_env
        return render_env(self._vec, 0)

    def close(self) -> None:
        self._vec.close()
