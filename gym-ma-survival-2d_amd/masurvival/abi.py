"""ctypes mirror of include/masurvival.h and the loader of the HIP library.

The product path is the HIP library ``libmas.so`` (built from ../csrc by
``__graft_entry__.build()``); there is no CPU fallback: :func:`load_library`
raises if the library is missing or cannot be loaded.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char, c_char_p, c_double, c_float, c_int32, c_int64, c_uint8,
                    c_uint64, c_void_p)

MAS_MAX_ZONE_PHASES = 8
MAS_MAX_KEYS = 16
MAS_STATS_WIDTH = 19
MAS_MAX_LASERS = 32


class MasConfig(Structure):
    _fields_ = [
        ('n_agents', c_int32), ('n_heals', c_int32), ('n_boxes', c_int32), ('teams', c_int32),
        ('ownership', c_int32), ('melee_cooldown', c_int32), ('omniscient', c_int32),
        ('gameover_mode', c_int32),
        ('r_alive', c_float), ('r_dead', c_float), ('r_kill', c_float), ('r_death', c_float),
        ('grid_size', c_int32), ('floor_size', c_double), ('agent_size', c_double),
        ('impulse', c_float * 3), ('agent_health', c_int32), ('melee_range', c_float),
        ('melee_damage', c_int32), ('box_size', c_double), ('box_health', c_int32),
        ('randomized_boxes', c_int32),
        ('avg_w', c_double), ('std_w', c_double), ('avg_h', c_double), ('std_h', c_double),
        ('min_w', c_double), ('min_h', c_double),
        ('box_item_size', c_double), ('box_item_offset', c_float), ('heal_size', c_double),
        ('healing', c_int32), ('slots', c_int32), ('pickup_radius', c_float), ('give_radius', c_float),
        ('deathdrop_radius', c_float), ('zone_phases', c_int32), ('zone_cooldown', c_int32),
        ('zone_damage', c_int32), ('zone_n_radii', c_int32), ('zone_radii', c_double * MAS_MAX_ZONE_PHASES),
        ('zone_random_centers', c_int32), ('zone_centers', (c_float * 2) * MAS_MAX_ZONE_PHASES),
        ('cam_depth', c_float), ('cam_fov', c_double), ('wall_aspect_ratio', c_double),
        ('lidar_n_lasers', c_int32), ('lidar_depth', c_float), ('lidar_fov', c_double),
    ]


class MasObsLayout(Structure):
    _fields_ = [
        ('n_agents', c_int32), ('obs_dim', c_int32), ('n_keys', c_int32),
        ('key_name', (c_char * 24) * MAS_MAX_KEYS), ('key_offset', c_int32 * MAS_MAX_KEYS),
        ('key_ndim', c_int32 * MAS_MAX_KEYS), ('key_shape', (c_int32 * 2) * MAS_MAX_KEYS),
    ]


# name -> (restype, argtypes); every symbol include/masurvival.h declares
SIGNATURES = {
    'mas_create': (c_int32, [POINTER(MasConfig), c_int64, c_int32, POINTER(c_void_p)]),
    'mas_destroy': (c_int32, [c_void_p]),
    'mas_get_obs_layout': (c_int32, [c_void_p, POINTER(MasObsLayout)]),
    'mas_num_envs': (c_int64, [c_void_p]),
    'mas_seed': (c_int32, [c_void_p, POINTER(c_uint64), c_void_p]),
    'mas_reset': (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'mas_step': (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    'mas_step_x': (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p]),
    'mas_step_x_supported': (c_int32, [c_void_p, c_int32]),
    'mas_flush_stats': (c_int32, [c_void_p, c_void_p, c_void_p]),
    'mas_state_bytes': (c_int64, [c_void_p]),
    'mas_get_state': (c_int32, [c_void_p, c_void_p, c_void_p]),
    'mas_set_state': (c_int32, [c_void_p, c_void_p, c_void_p]),
    'mas_gae': (c_int32, [c_int32, c_int64, c_int32, c_void_p, c_void_p, c_void_p, ctypes.c_float, ctypes.c_float,
                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'mas_gae_scratch_doubles': (c_int64, [c_int64]),
    'mas_adv_normalize': (c_int32, [c_int64, c_void_p, c_void_p, c_void_p]),
    'mas_debug_counters': (c_int32, [c_void_p, POINTER(c_int64)]),
    'mas_debug_guards': (c_int32, [c_void_p, POINTER(c_int64)]),
    'mas_debug_force_general': (c_int32, [c_void_p, c_int32]),
    'mas_invalid_actions': (c_int32, [c_void_p, POINTER(c_int64), c_int32]),
    'mas_debug_gen_flags': (c_int32, [c_void_p, c_void_p, c_void_p]),
    'mas_debug_set_toi_counter': (c_int32, [c_void_p, c_void_p]),
    'mas_sample_actions': (c_int32, [c_int64, c_void_p, c_int64, ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_void_p,
                                     c_void_p]),
    'mas_render_view': (c_int32, [c_void_p, c_int64, c_void_p]),
    'mas_policy_packed_bytes': (c_int64, [c_int32]),
    'mas_policy_blocks': (c_int64, [c_int64]),
    'mas_policy_pack': (c_int32, [c_int32] + [c_void_p] * 8),
    'mas_policy_act': (c_int32, [c_void_p, c_int32, c_int64, c_void_p, c_void_p, c_int64, ctypes.c_uint64,
                                 ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    'mas_policy_act_rows': (c_int32, [c_void_p, c_int32, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                      ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    'mas_policy_act_x': (c_int32, [c_void_p, c_int32, c_int64, c_int64, c_void_p, c_int64, ctypes.c_uint64,
                                   ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    'mas_policy_train': (c_int32, [c_void_p, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                   c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float]
                         + [c_void_p] * 7),
    'mas_policy_train_ld': (c_int32, [c_void_p, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                      c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float]
                            + [c_void_p] * 5 + [c_int64, c_void_p, c_void_p]),
    'mas_policy_train_rm': (c_int32, [c_void_p, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                      c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float]
                            + [c_void_p, c_void_p, c_int64] + [c_void_p] * 5),
    'mas_policy_rm_feature': (c_int32, [c_int32]),
    'mas_policy_adam_scratch': (c_int64, []),
    'mas_policy_adam': (c_int32, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float, ctypes.c_float,
                                  c_double, c_double, c_double, c_double, c_int64, c_void_p, c_void_p]),
    'mas_policy_dw_scratch': (c_int64, [c_int32, c_int32, c_int64]),
    'mas_policy_dw': (c_int32, [c_int32, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                c_void_p]),
    'mas_last_error': (c_char_p, []),
    'mas_abi_version': (c_int32, []),
}

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# MAS_LIB: an alternative build of the library (A/B variants, libmas_<name>.so)
LIB_PATH = os.environ.get('MAS_LIB') or os.path.join(PKG_DIR, '_lib', 'libmas.so')

_lib = None


class MasError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libmas.so (the HIP product path).  Fails loudly when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MasError(f'HIP extension not built: {path} missing (run __graft_entry__.build())')
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.mas_last_error().decode() if _lib is not None else ''
        raise MasError(f'masurvival C-ABI error {rc}: {msg}')
