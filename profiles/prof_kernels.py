"""Per-phase wave time of k_pre, k_post and k_obs from the profiling build
(libmas_prof.so, `make -C gym-ma-survival-2d_amd/csrc prof`): the first
active lane of each wave adds the 100 MHz constant-clock time since the
previous mark (MAS_PROF, mas_kernels.inc marks 30..40).  Printed: the mean
per wave per step (us).  The envs run the PPO trainer's regime (2 warm-up
iterations, then rollout steps of the trained policy), as the headline bench.
usage: python profiles/prof_kernels.py [n_envs] [steps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import torch  # noqa: E402,F401

from masurvival import abi  # noqa: E402

MARKS = {30: 'k_pre: state load', 41: 'k_pre: step_pre queue_actions', 42: 'k_pre: step_pre drops + motors',
         43: 'k_pre: step_pre UseLast', 44: 'k_pre: step_pre GiveLast', 45: 'k_pre: step_pre melee fixtab + jobs',
         46: 'k_pre: step_pre melee ray casts', 31: 'k_pre: step_pre melee attacks (rest)', 32: 'k_pre: dirty stores',
         33: 'k_pre: contact-free fast physics', 34: 'k_post: state load', 35: 'k_post: step_post',
         36: 'k_post: stores', 37: 'k_obs: auto-reset', 38: 'k_obs: state load', 39: 'k_obs: row writer (windows)',
         40: 'k_obs: tile stores (windows)'}
WAVES = {'k_pre': 1024, 'k_post': 1024, 'k_obs': 4096}  # 2v2 x65536


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.ppo import PPOConfig, PPOTrainer
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(), seed=0)
    for _ in range(2):
        tr.iteration()
    buf = (ctypes.c_ulonglong * 64)()
    abi.check(lib.mas_prof_read(env._h, buf))
    for t in range(steps):
        tr.rollout_step(t)
    abi.check(lib.mas_prof_read(env._h, buf))
    scale = n / 65536
    for k, name in MARKS.items():
        w = WAVES[name.split(':')[0]] * scale
        print(f'{name:42s} {buf[k] * 0.01 / (w * steps):8.2f} us per wave')


if __name__ == '__main__':
    main()
