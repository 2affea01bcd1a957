"""TEST INFRASTRUCTURE: generate the golden episode fixtures tests/golden/*.npz.

Runs the REFERENCE's own Python -- masurvival/simulation.py, semantics.py and
envs/masurvival_env.py from /root/reference, compiled here from their source
text (the reference's shipped __pycache__ is never read; no bytecode is
written) -- over tests/golden/shim: test-only Box2D/gym stand-ins whose
geometry/physics is the C oracle (oracle/build/libmas_oracle.so).

What this pins: the oracle's restatement of the reference's game rules,
module order, spawn/despawn list order, RNG use, observation assembly,
rewards, done and stats is checked against the reference code itself
(tests/test_golden.py replays each fixture through the C oracle and requires
bit-identical obs / rewards / done).  What it does not pin: Box2D's own
arithmetic (PyBox2D is absent; the shim uses the oracle's physics).

Fixtures are data only: actions, reset/step observations (flattened in
observation_space key order), rewards, done, stats, seeds and the config.
Usage:  python tests/golden/make_golden.py   (needs /root/reference)
"""
from __future__ import annotations

import copy
import json
import math
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('MAS_REFERENCE', '/root/reference')
sys.path.insert(0, os.path.join(HERE, 'shim'))

import Box2D  # noqa: E402  (the shim)


def load_reference():
    """Import the reference package from source text under its own name
    (this process never imports the product's ``masurvival``)."""
    pkg = types.ModuleType('masurvival')
    pkg.__path__ = []
    envs = types.ModuleType('masurvival.envs')
    envs.__path__ = []
    sys.modules['masurvival'] = pkg
    sys.modules['masurvival.envs'] = envs
    pkg.envs = envs
    for name, rel, parent, leaf in [
        ('masurvival.simulation', 'masurvival/simulation.py', pkg, 'simulation'),
        ('masurvival.semantics', 'masurvival/semantics.py', pkg, 'semantics'),
        ('masurvival.envs.masurvival_env', 'masurvival/envs/masurvival_env.py', envs, 'masurvival_env'),
    ]:
        path = os.path.join(REF, rel)
        with open(path) as fh:
            src = fh.read()
        mod = types.ModuleType(name)
        mod.__file__ = path
        sys.modules[name] = mod
        setattr(parent, leaf, mod)
        exec(compile(src, path, 'exec'), mod.__dict__)
    return sys.modules['masurvival.envs.masurvival_env']


def flatten_obs(obs):
    keys = sorted(obs.keys())
    A = obs['agent'].shape[0]
    return np.concatenate([np.asarray(obs[k], dtype=np.float32).reshape(A, -1) for k in keys], axis=1), keys


def scripted_actions(obs, rng, A, p_script, teams):
    """Mix of uniform-random and two scripted roles, to exercise fights,
    kills, death drops, pickups, use/give and box break/placement:
    even agents hunt the nearest opponent, odd agents go for the nearest box
    or box item (break it, pick the item up, place it again)."""
    acts = []
    ag = obs['agent']
    o = 1 if teams else 0
    for i in range(A):
        a = rng.integers(0, [3, 3, 3, 2, 2, 2])
        if rng.random() < p_script and ag[i][1 + o] > 0:
            x, y, th = ag[i][2 + o], ag[i][3 + o], ag[i][4 + o]
            targets = []
            if i % 2 == 0 or 'boxes' not in obs:
                for j in range(A):
                    if j == i or ag[j][1 + o] <= 0 or (teams and ag[j][1] == ag[i][1]):
                        continue
                    targets.append((ag[j][2 + o], ag[j][3 + o], 'agent'))
            else:
                for b in range(obs['boxes'].shape[1]):
                    if obs['boxes_mask'][i][b] == 0:
                        targets.append((obs['boxes'][i][b][8], obs['boxes'][i][b][9], 'box'))
                for b in range(obs['box_items'].shape[1]):
                    if obs['box_items_mask'][i][b] == 0:
                        targets.append((obs['box_items'][i][b][8], obs['box_items'][i][b][9], 'item'))
            best, bd = None, 1e9
            for tx, ty, kind in targets:
                d = math.hypot(tx - x, ty - y)
                if d < bd:
                    best, bd = (tx, ty, kind), d
            if best is not None:
                phi = math.atan2(best[1] - y, best[0] - x)
                dl = (phi - th + math.pi) % (2 * math.pi) - math.pi
                a[2] = 2 if dl > 0.15 else (0 if dl < -0.15 else 1)
                a[0] = 2 if (abs(dl) < 0.6 and (best[2] != 'box' or bd > 1.2)) else 1
                a[3] = 1 if (bd < 2.4 and best[2] != 'item') else int(rng.random() < 0.2)
            has_box = 'box_slot_mask' in obs and obs['box_slot_mask'][i][0] == 0
            a[4] = int(rng.random() < (0.5 if has_box else 0.3))
            a[5] = int(rng.random() < 0.15)
        acts.append(a.astype(np.int64))
    return tuple(acts)


def collector_actions(obs, rng, A, teams):
    """Walk over the nearest heal / box item, never use; give often -- fills
    inventories (lost gives), makes agents converge on the same item (double
    pickups) and die carrying items (death drops)."""
    acts = []
    ag = obs['agent']
    o = 1 if teams else 0
    for i in range(A):
        a = rng.integers(0, [3, 3, 3, 2, 2, 2])
        a[4] = 0
        if ag[i][1 + o] > 0:
            x, y, th = ag[i][2 + o], ag[i][3 + o], ag[i][4 + o]
            targets = []
            if 'heals' in obs:
                for h in range(obs['heals'].shape[1]):
                    if obs['heals_mask'][i][h] == 0:
                        targets.append((obs['heals'][i][h][0], obs['heals'][i][h][1]))
            if 'box_items' in obs:
                for b in range(obs['box_items'].shape[1]):
                    if obs['box_items_mask'][i][b] == 0:
                        targets.append((obs['box_items'][i][b][8], obs['box_items'][i][b][9]))
            if targets and rng.random() < 0.85:
                tx, ty = min(targets, key=lambda p: math.hypot(p[0] - x, p[1] - y))
                phi = math.atan2(ty - y, tx - x)
                dl = (phi - th + math.pi) % (2 * math.pi) - math.pi
                a[2] = 2 if dl > 0.15 else (0 if dl < -0.15 else 1)
                a[0] = 2 if abs(dl) < 0.6 else 1
                a[1] = 1
            a[3] = int(rng.random() < 0.3)
            a[5] = int(rng.random() < 0.4)
        acts.append(a.astype(np.int64))
    return tuple(acts)


def hoarder_actions(obs, rng, A, teams):
    """Walk over the nearest heal / box item and keep it: never use, give
    rarely, attack rarely -- inventories fill past four slots (the ffal
    capacity class: Inventory with slots > 4, semantics.py:165-245)."""
    acts = collector_actions(obs, rng, A, teams)
    out = []
    for a in acts:
        a = a.copy()
        a[3] = int(rng.random() < 0.05)
        a[5] = int(rng.random() < 0.03)
        out.append(a)
    return tuple(out)


def max_inventory(env):
    """Longest inventory list of any agent right now (Inventory.inventories)."""
    sem = sys.modules['masurvival.semantics']
    invs = env.simulation.groups['agents'].get(sem.Inventory)
    return max((len(v) for m in invs for v in m.inventories.values()), default=0)


def lidar_obs(env, lidars):
    """The 'lidars' observation key of this build: the
    reference's own Lidars module (simulation.py:357-392) computes the scans;
    agent i's row holds its lasers' relative depths (laser_scan :431-439), 1
    where nothing is hit, zeros for a dead agent (no body).  Lidars is the
    last agents module, so scans[k] belongs to agents.bodies[k]."""
    agents = env.simulation.groups['agents']
    sim = sys.modules['masurvival.simulation']
    indexed = agents.get(sim.IndexBodies)[0].bodies
    out = np.zeros((env.n_agents, lidars.n_lasers), dtype=np.float32)
    for i, body in enumerate(indexed):
        if body is None:
            continue
        k = agents.bodies.index(body)
        out[i] = [1.0 if s is None else s[1] for s in lidars.scans[k]]
    return out


def run_episode(mod, name, config, env_seed, act_seed, max_steps, p_script):
    lid_cfg = None
    if config is not None and 'lidars' in config:
        # the reference env has no 'lidars' config key (BaseEnv merge raises
        # KeyError); its Lidars module is attached as the last agents module
        config = dict(config)
        lid_cfg = config.pop('lidars')
    env = mod.MaSurvival(config=copy.deepcopy(config) if config is not None else None)
    lidars = None
    if lid_cfg is not None:
        sim = sys.modules['masurvival.simulation']
        lidars = sim.Lidars(**lid_cfg)
        env.simulation.groups['agents'].modules.append(lidars)
        config = dict(config, lidars=lid_cfg)
    groups = env.simulation.groups
    Box2D.CANONICAL_GROUPS[:] = list(groups.values())
    Box2D.STATIC_GROUPS[:] = [groups['walls'], groups['boxes']]
    env.np_random = np.random.default_rng(env_seed)
    obs = env.reset()
    if lidars is not None:
        obs['lidars'] = lidar_obs(env, lidars)
    flat0, keys = flatten_obs(obs)
    A = env.n_agents
    rng = np.random.default_rng(act_seed)
    obs_l, act_l, rew_l, done_l = [flat0], [], [], []
    max_inv = 0
    for t in range(max_steps):
        if p_script == -1:  # idle stretches (Box2D sleep): no-op except a random burst every 150 steps
            acts = tuple(np.array([1, 1, 1, 0, 0, 0]) if (t % 150) > 3 else rng.integers(0, [3, 3, 3, 2, 2, 2])
                         for _ in range(A))
        elif p_script == -2:
            acts = collector_actions(obs, rng, A, env.has_teams)
        elif p_script == -3:
            acts = hoarder_actions(obs, rng, A, env.has_teams)
        else:
            acts = scripted_actions(obs, rng, A, p_script, env.has_teams)
        obs, rew, done, info = env.step(acts)
        if lidars is not None:
            obs['lidars'] = lidar_obs(env, lidars)
        obs_l.append(flatten_obs(obs)[0])
        act_l.append(np.stack(acts).astype(np.int8))
        rew_l.append(np.asarray(rew, dtype=np.float32))
        done_l.append(bool(done))
        max_inv = max(max_inv, max_inventory(env))
        if done:
            break
    stats = env.flush_stats()
    return dict(
        name=name,
        config=json.dumps(config),
        env_seed=env_seed,
        act_seed=act_seed,
        keys=json.dumps(keys),
        obs=np.stack(obs_l).astype(np.float32),
        actions=np.stack(act_l),
        rewards=np.stack(rew_l),
        done=np.array(done_l, dtype=np.bool_),
        stats=json.dumps({k: float(v) for k, v in stats.items()}),
        max_inventory=np.int32(max_inv),
    )


MELEE = {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}
EPISODES = [
    # name, config (JSON-able; None = class default), env seed, action seed, max steps, p_script
    ('c1_random_s0', None, 0, 100, 1000, 0.0),
    ('c1_script_s1', None, 1, 101, 1000, 0.8),
    ('c1_script_s2', {'melee': MELEE, 'reward_scheme': {'r_alive': 1, 'r_dead': -1, 'r_kill': 5, 'r_death': -5}},
     2, 102, 1000, 0.9),
    ('c3_2v2_script_s3', {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True}, 'melee': MELEE,
                          'reward_scheme': {'r_alive': 1, 'r_dead': -1, 'r_kill': 3, 'r_death': -2}},
     3, 103, 1000, 0.8),
    ('c3_2v2_random_s4', {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True}, 'melee': MELEE},
     4, 104, 400, 0.0),
    ('c5_ffa4_script_s5', {
        'agents': {'n_agents': 4, 'agent_size': 1},
        'spawn_grid': {'grid_size': 8, 'floor_size': 20},
        'heals': {'reset_spawns': {'n_items': 16, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': False,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
                  'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
        'melee': MELEE,
        'reward_scheme': {'r_alive': 1, 'r_dead': -1, 'r_kill': 2, 'r_death': 0}}, 5, 105, 1000, 0.7),
    ('ownership_contmelee_s6', {
        'agents': {'n_agents': 3, 'agent_size': 1},
        'boxes': {'reset_spawns': {'n_boxes': 6, 'box_size': 1}, 'ownership': True,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
        'melee': {'range': 2, 'damage': 5, 'drift': True}}, 6, 106, 700, 0.8),
    ('nonomni_lastalive_s7', {
        'agents': {'n_agents': 4, 'agent_size': 1}, 'observation': {'omniscent': False},
        'gameover': {'mode': 'lastalive'}, 'melee': MELEE}, 7, 107, 1000, 0.8),
    ('idle_sleep_s9', {'melee': MELEE, 'safe_zone': {'phases': 5, 'cooldown': 150, 'damage': 1,
                                                      'radiuses': [40, 30, 20, 10], 'centers': 'random'}},
     9, 109, 700, -1),
    ('collect_ffa4_s10', {
        'agents': {'n_agents': 4, 'agent_size': 1},
        'spawn_grid': {'grid_size': 6, 'floor_size': 20},
        'heals': {'reset_spawns': {'n_items': 12, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 8, 'box_size': 1}, 'ownership': False,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
        'inventory': {'slots': 3},
        'melee': MELEE}, 10, 110, 1000, -2),
    ('collect_2v2_s11', {
        'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True},
        'spawn_grid': {'grid_size': 6, 'floor_size': 20},
        'heals': {'reset_spawns': {'n_items': 10, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'melee': MELEE}, 11, 111, 1000, -2),
    ('noheals_noboxes_s8', {
        'heals': {'reset_spawns': {'n_items': 0, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 0, 'box_size': 1}, 'ownership': False,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
        'melee': MELEE}, 8, 108, 300, 0.5),
    # Lidars (simulation.py:357-392), opt-in 'lidars' key: 2v2 fights, FFA4
    # with heals + randomized boxes (rays hit every body kind), and the
    # minimum of two lasers with rays longer than the room
    ('lidars_2v2_s12', {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True}, 'melee': MELEE,
                        'lidars': {'n_lasers': 8, 'fov': 0.5 * math.pi, 'depth': 6}}, 12, 112, 600, 0.8),
    ('lidars_ffa4_s13', {
        'agents': {'n_agents': 4, 'agent_size': 1},
        'spawn_grid': {'grid_size': 6, 'floor_size': 14},
        'heals': {'reset_spawns': {'n_items': 8, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 8, 'box_size': 1}, 'ownership': False,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
                  'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
        'melee': MELEE, 'lidars': {'n_lasers': 16, 'fov': 2.0 * math.pi * 15 / 16, 'depth': 5.5}},
     13, 113, 500, -2),
    ('lidars_1v1_s14', {'melee': MELEE, 'lidars': {'n_lasers': 2, 'fov': 0.3, 'depth': 30}}, 14, 114, 400, 0.6),
    # the ffal capacity class (more than 16 heals or 4 slots): hoarders fill
    # inventories past four slots (max_inventory > 4 is asserted by the tests)
    ('ffal_ffa4_s15', {
        'agents': {'n_agents': 4, 'agent_size': 1},
        'spawn_grid': {'grid_size': 6, 'floor_size': 16},
        'heals': {'reset_spawns': {'n_items': 20, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 12, 'box_size': 1}, 'ownership': False,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
                  'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
        'inventory': {'slots': 6},
        'safe_zone': {'phases': 5, 'cooldown': 200, 'damage': 1, 'radiuses': [16, 8, 4, 2], 'centers': 'random'},
        'melee': MELEE}, 15, 115, 1200, -3),
    ('ffal_2v2_owned_s16', {
        'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True},
        'spawn_grid': {'grid_size': 7, 'floor_size': 18},
        'heals': {'reset_spawns': {'n_items': 24, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': True,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
        'inventory': {'slots': 8},
        'safe_zone': {'phases': 5, 'cooldown': 200, 'damage': 1, 'radiuses': [16, 8, 4, 2], 'centers': 'random'},
        'melee': MELEE}, 16, 116, 1200, -3),
    # the xxl capacity class (5-8 agents with up to 20 heals, 16 boxes, 8
    # slots): eight hoarders in a free-for-all; a 4v4 fight with owned boxes
    ('xxl_ffa8_s17', {
        'agents': {'n_agents': 8, 'agent_size': 1},
        'spawn_grid': {'grid_size': 8, 'floor_size': 22},
        'heals': {'reset_spawns': {'n_items': 20, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': False,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
                  'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
        'inventory': {'slots': 8},
        'safe_zone': {'phases': 5, 'cooldown': 200, 'damage': 1, 'radiuses': [22, 11, 5, 2], 'centers': 'random'},
        'melee': MELEE}, 17, 117, 1200, -3),
    ('xxl_4v4_owned_s18', {
        'agents': {'n_agents': 8, 'agent_size': 1}, 'teams': {'twoteams': True},
        'spawn_grid': {'grid_size': 7, 'floor_size': 20},
        'heals': {'reset_spawns': {'n_items': 16, 'item_size': 0.5}, 'heal': {'healing': 50}},
        'boxes': {'reset_spawns': {'n_boxes': 12, 'box_size': 1}, 'ownership': True,
                  'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
        'inventory': {'slots': 6},
        'melee': MELEE,
        'reward_scheme': {'r_alive': 1, 'r_dead': -1, 'r_kill': 3, 'r_death': -2}}, 18, 118, 1000, 0.8),
]


def main(only=None):
    for name, config, es, as_, T, p in EPISODES:
        if only and name not in only:
            continue
        # fresh import per episode: MaSurvival(config=None) mutates the
        # class-level default config (masurvival_env.py:51-54 share nested
        # dicts, :301/:348/:371 pop from them), so a second construction in
        # one process raises KeyError('box_size').
        mod = load_reference()
        d = run_episode(mod, name, config, es, as_, T, p)
        out = os.path.join(HERE, name + '.npz')
        np.savez_compressed(out, **d)
        print(f"{name}: steps={len(d['done'])} done={bool(d['done'][-1])} max_inv={int(d['max_inventory'])} "
              f"stats={d['stats']} "
              f"-> {os.path.getsize(out) // 1024} KiB", flush=True)


if __name__ == '__main__':
    main(sys.argv[1:])
