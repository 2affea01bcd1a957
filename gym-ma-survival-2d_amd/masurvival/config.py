"""Env configuration front-end.

Mirrors the reference's config handling exactly:
  * ``onevsone_heals_config`` defaults  (masurvival/envs/masurvival_env.py:140-238)
  * deep copy + one-level merge ``self.config[k] |= subconfig`` with KeyError on
    unknown top-level keys                   (masurvival_env.py:49-56, 909-918)
  * ``'cooldown' in config['melee']`` of the USER config selects Melee vs
    ContinuousMelee                          (masurvival_env.py:309-312)
and lowers the merged dict to the POD ``mas_config`` consumed by the C-ABI
(include/masurvival.h).  Shapes in the reference config (auto_pickup / give)
are b2CircleShape objects; here any object with a ``radius`` attribute (see
:func:`circle_shape`) or a plain number is accepted.
"""
from __future__ import annotations

import copy
import math
from typing import Any, Dict, Optional

import numpy as np

from .abi import MAS_MAX_LASERS, MAS_MAX_ZONE_PHASES, MasConfig


class CircleShape:
    """Stand-in for ``b2CircleShape(radius=r)`` in config dicts (simulation.py:59-60)."""

    def __init__(self, radius: float):
        self.radius = float(radius)

    def __repr__(self):
        return f"circle_shape({self.radius})"

    def __deepcopy__(self, memo):
        return CircleShape(self.radius)


def circle_shape(radius: float) -> CircleShape:
    return CircleShape(radius)


onevsone_heals_config: Dict[str, Dict[str, Any]] = {
    'observation': {'omniscent': True},
    'reward_scheme': {'r_alive': 1, 'r_dead': -1, 'r_kill': 0, 'r_death': 0},
    'gameover': {'mode': 'alldead'},
    'rng': {'seed': 42},
    'spawn_grid': {'grid_size': 4, 'floor_size': 20},
    'immunity_phase': {'cooldown': 300},
    'agents': {'n_agents': 2, 'agent_size': 1},
    'teams': {'twoteams': False},
    'cameras': {'fov': 0.4 * np.pi, 'depth': 10},
    'motors': {'impulse': (0.25, 0.25, 0.0125), 'drift': False},
    'health': {'health': 100},
    'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True},
    'boxes': {
        'reset_spawns': {'n_boxes': 4, 'box_size': 1},
        'ownership': False,
        'item': {'item_size': 0.5, 'offset': 0.75},
        'health': 20,
    },
    'heals': {
        'reset_spawns': {'n_items': 4, 'item_size': 0.5},
        'heal': {'healing': 50},
    },
    'inventory': {'slots': 4},
    'auto_pickup': {'shape': circle_shape(0.5)},
    'give': {'shape': circle_shape(2)},
    'death_drop': {'radius': 0.5},
    'safe_zone': {
        'phases': 5,
        'cooldown': 100,
        'damage': 1,
        'radiuses': [10, 5, 2.5, 1],
        'centers': 'random',
    },
}


def merge_config(user_config: Optional[Dict[str, Dict[str, Any]]]) -> Dict[str, Dict[str, Any]]:
    """BaseEnv.__init__ merge (masurvival_env.py:49-56): deep copy of the
    defaults, then ``self.config[k] |= subconfig`` -- unknown top-level keys
    raise KeyError and nested sub-dicts are replaced, not merged."""
    config = copy.deepcopy(onevsone_heals_config)
    if user_config is not None:
        for k, sub in user_config.items():
            if k == 'lidars':
                # extension key: the reference defines Lidars
                # (simulation.py:357-392) but never wires it into the env
                # (masurvival_env.py:392, 857-858); here it is opt-in
                config[k] = dict(sub)
                continue
            config[k] |= sub  # KeyError on unknown k, as in the reference
    return config


def _radius(shape_or_r: Any) -> float:
    if hasattr(shape_or_r, 'radius'):
        return float(shape_or_r.radius)
    return float(shape_or_r)


def _pick(d: Dict[str, Any], *keys: str) -> Any:
    for k in keys:
        if k in d and d[k] is not None:
            return d[k]
    raise KeyError(keys[0])


class ResolvedConfig:
    """The merged config plus the derived facts MaSurvival.__init__ computes."""

    def __init__(self, user_config: Optional[Dict[str, Dict[str, Any]]] = None):
        if user_config is None:
            user_config = onevsone_heals_config
        self.user_config = user_config
        self.config = merge_config(user_config)
        c = self.config
        # MaSurvival.__init__ reads config['melee'] of the USER config (:310)
        self.continuous_melee = 'cooldown' not in user_config['melee']
        self.n_agents = int(c['agents'].get('n_spawns', None) or c['agents']['n_agents'])
        self.n_heals = int(_pick(c['heals']['reset_spawns'], 'n_items', 'n_spawns'))
        self.n_boxes = int(_pick(c['boxes']['reset_spawns'], 'n_boxes', 'n_spawns'))
        self.has_teams = 'teams' in c and bool(c['teams']['twoteams'])
        self.box_ownership = bool(c.get('boxes', {}).get('ownership', False))
        if self.n_agents < 2:
            # np.concatenate([]) in fetch_observations (masurvival_env.py:529-534)
            raise ValueError('n_agents must be >= 2 (the reference crashes building others obs)')
        g = int(c['spawn_grid']['grid_size'])
        if self.n_agents + self.n_heals + self.n_boxes > g * g:
            raise IndexError('pop from empty list: more spawns than spawn-grid cells (semantics.py:77)')
        if c['gameover']['mode'] not in ('alldead', 'lastalive'):
            raise AssertionError('Invalid gameover mode')
        self.lidars = c.get('lidars')
        if self.lidars is not None:
            n = int(self.lidars['n_lasers'])
            if not 2 <= n <= MAS_MAX_LASERS:
                # n_lasers = 1 divides by zero in Lidars._endpoints (simulation.py:388)
                raise ValueError(f'lidars.n_lasers must be in [2, {MAS_MAX_LASERS}]')

    @property
    def agent_size(self) -> int:
        return 8 + (1 if self.has_teams else 0)

    def to_struct(self) -> MasConfig:
        c = self.config
        s = MasConfig()
        s.n_agents = self.n_agents
        s.n_heals = self.n_heals
        s.n_boxes = self.n_boxes
        s.teams = int(self.has_teams)
        s.ownership = int(self.box_ownership)
        s.melee_cooldown = 0 if self.continuous_melee else int(c['melee']['cooldown'])
        s.omniscient = int(bool(c['observation']['omniscent']))
        s.gameover_mode = 0 if c['gameover']['mode'] == 'alldead' else 1
        rs = c['reward_scheme']
        s.r_alive = float(rs.get('r_alive', 0))
        s.r_dead = float(rs.get('r_dead', 0))
        s.r_kill = float(rs.get('r_kill', 0))
        s.r_death = float(rs.get('r_death', 0))
        s.grid_size = int(c['spawn_grid']['grid_size'])
        s.floor_size = float(c['spawn_grid']['floor_size'])
        s.agent_size = float(c['agents']['agent_size'])
        imp = c['motors']['impulse']
        for k in range(3):
            s.impulse[k] = float(imp[k])
        s.agent_health = int(c['health']['health'])
        s.melee_range = float(c['melee']['range'])
        s.melee_damage = int(c['melee']['damage'])
        bcfg = c['boxes']
        s.box_size = float(bcfg['reset_spawns'].get('box_size', 1))
        s.box_health = int(bcfg['health'])
        if 'randomized_shape' in bcfg:
            r = bcfg['randomized_shape']
            s.randomized_boxes = 1
            s.avg_w, s.std_w = float(r['avg_w']), float(r['std_w'])
            s.avg_h, s.std_h = float(r['avg_h']), float(r['std_h'])
            s.min_w, s.min_h = float(r.get('min_w', 0.1)), float(r.get('min_h', 0.1))
        else:
            s.min_w = s.min_h = 0.1
        s.box_item_size = float(bcfg['item']['item_size'])
        s.box_item_offset = float(bcfg['item']['offset'])
        hcfg = c['heals']
        s.heal_size = float(hcfg['reset_spawns']['item_size'])
        s.healing = int(hcfg['heal']['healing'])
        s.slots = int(c['inventory']['slots'])
        s.pickup_radius = _radius(c['auto_pickup']['shape'])
        s.give_radius = _radius(c['give']['shape'])
        s.deathdrop_radius = float(c['death_drop']['radius'])
        z = c['safe_zone']
        s.zone_phases = int(z['phases'])
        s.zone_cooldown = int(z['cooldown'])
        s.zone_damage = int(z['damage'])
        radii = list(z['radiuses'])
        if len(radii) + 1 > MAS_MAX_ZONE_PHASES or s.zone_phases > len(radii) + 1:
            raise ValueError('safe_zone: at most %d phases supported' % (MAS_MAX_ZONE_PHASES - 1))
        s.zone_n_radii = len(radii)
        for k, r in enumerate(radii):
            s.zone_radii[k] = float(r)
        if z['centers'] == 'random':
            s.zone_random_centers = 1
        else:
            s.zone_random_centers = 0
            for k, cc in enumerate(z['centers']):
                s.zone_centers[k][0] = float(cc[0])
                s.zone_centers[k][1] = float(cc[1])
        s.cam_depth = float(c['cameras']['depth'])
        s.cam_fov = float(c['cameras']['fov'])
        s.wall_aspect_ratio = 100.0
        if self.lidars is not None:
            s.lidar_n_lasers = int(self.lidars['n_lasers'])
            s.lidar_fov = float(self.lidars['fov'])
            s.lidar_depth = float(self.lidars['depth'])
        return s


# Named benchmark / parity configurations.
C1_CONFIG: Dict[str, Dict[str, Any]] = {'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}}
C3_CONFIG: Dict[str, Dict[str, Any]] = {
    'agents': {'n_agents': 4, 'agent_size': 1},
    'teams': {'twoteams': True},
    'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True},
}
C5_CONFIG: Dict[str, Dict[str, Any]] = {
    'agents': {'n_agents': 4, 'agent_size': 1},
    'spawn_grid': {'grid_size': 8, 'floor_size': 20},
    'heals': {'reset_spawns': {'n_items': 16, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {
        'reset_spawns': {'n_boxes': 16, 'box_size': 1},
        'ownership': False,
        'item': {'item_size': 0.5, 'offset': 0.75},
        'health': 20,
        'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5},
    },
    'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True},
}
NAMED_CONFIGS = {'1v1': C1_CONFIG, '2v2': C3_CONFIG, 'ffa4': C5_CONFIG}


def pcg64_state(seed: int) -> np.ndarray:
    """numpy ``default_rng(seed)`` bit-generator state as the 6 uint64 words
    the C-ABI takes (masurvival_env.py:50: one Generator per env)."""
    st = np.random.PCG64(seed).state
    s, inc = int(st['state']['state']), int(st['state']['inc'])
    m = (1 << 64) - 1
    return np.array([s >> 64, s & m, inc >> 64, inc & m, int(st['has_uint32']), int(st['uinteger'])],
                    dtype=np.uint64)
