"""Import shim: exposes the package directory
``drone-2d-custom-gym-env-for-reinforcement-learning_amd/`` (not a valid identifier) as the
module ``drone2d_amd``, with working relative imports of its submodules."""
import importlib.util as _iu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                         "drone-2d-custom-gym-env-for-reinforcement-learning_amd")
_spec = _iu.spec_from_file_location(__name__, _os.path.join(_PKG_DIR, "__init__.py"),
                                    submodule_search_locations=[_PKG_DIR])
_mod = _iu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
