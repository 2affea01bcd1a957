"""Observation layout: compute_obs_space (masurvival_env.py:391-447) as a flat
per-agent row.  Keys follow gym-0.21 ``spaces.Dict`` order (sorted), each
key's per-agent sub-array is flattened C-order.  This is the same layout the
HIP kernels write (checked against mas_get_obs_layout in the tests)."""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Tuple


def obs_key_shapes(n_agents: int, n_heals: int, n_boxes: int, has_teams: bool,
                   n_lasers: int = 0) -> 'OrderedDict[str, Tuple[int, ...]]':
    """Per-agent sub-array shape for every observation key, in Dict order.
    ``n_lasers`` > 0 adds the opt-in 'lidars' key (one relative depth per
    laser of the Lidars module, simulation.py:357-392)."""
    agent_size = 1 + 1 + 3 + 3 + (1 if has_teams else 0)
    d: Dict[str, Tuple[int, ...]] = {
        'agent': (agent_size,),
        'zone': (6,),
        'others': (n_agents - 1, agent_size),
        'others_mask': (n_agents - 1,),
    }
    if n_heals > 0:
        d['heals'] = (n_heals, 2)
        d['heals_mask'] = (n_heals,)
        d['heal_slot'] = (1, 1)
        d['heal_slot_mask'] = (1,)
    if n_boxes > 0:
        d['boxes'] = (n_boxes, 11)
        d['boxes_mask'] = (n_boxes,)
        d['box_items'] = (n_boxes, 10)
        d['box_items_mask'] = (n_boxes,)
        d['box_slot'] = (1, 8)
        d['box_slot_mask'] = (1,)
    if n_lasers > 0:
        d['lidars'] = (n_lasers,)
    return OrderedDict(sorted(d.items()))


def obs_layout(n_agents: int, n_heals: int, n_boxes: int, has_teams: bool, n_lasers: int = 0):
    """Returns (obs_dim, {key: (offset, per-agent shape)})."""
    off = 0
    out = OrderedDict()
    for k, shp in obs_key_shapes(n_agents, n_heals, n_boxes, has_teams, n_lasers).items():
        size = 1
        for s in shp:
            size *= s
        out[k] = (off, shp)
        off += size
    return off, out


def split_obs(flat, layout):
    """Slice a [..., A, D] array/tensor into the reference obs dict (views)."""
    out = OrderedDict()
    for k, (off, shp) in layout.items():
        size = 1
        for s in shp:
            size *= s
        out[k] = flat[..., off:off + size].reshape(*flat.shape[:-1], *shp)
    return out
