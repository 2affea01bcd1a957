"""TEST-ONLY stand-in for gym 0.21 (absent from this image): just gym.Env and
gym.spaces, re-exported from the product's gym-0.21-compatible spaces."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_p = _os.path.abspath(_os.path.join(_os.path.dirname(__file__), '..', '..', '..', '..',
                                    'gym-ma-survival-2d_amd', 'masurvival', 'spaces.py'))
_spec = _ilu.spec_from_file_location('gym.spaces', _p)
spaces = _ilu.module_from_spec(_spec)
_spec.loader.exec_module(spaces)
_sys.modules['gym.spaces'] = spaces


class Env:
    pass
