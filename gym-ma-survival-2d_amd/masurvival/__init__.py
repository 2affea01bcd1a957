"""masurvival -- MI355X-native batched MaSurvival (KRLGroup/gym-ma-survival-2d).

The env step runs as hand-written HIP kernels (libmas.so, C-ABI in
include/masurvival.h).  The import path ``masurvival.envs.masurvival_env`` of
the reference (demo.py:11) is kept; ``masurvival.vec_env.VecMaSurvival`` is
the batched surface.
"""
__version__ = '0.1.0'
