"""Import alias: the package lives in the hyphenated directory ``gym-treasure-game_amd/``.

``import gym_treasure_game_amd`` loads that directory as the package of this name (its
submodules resolve there too).
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "gym-treasure-game_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
