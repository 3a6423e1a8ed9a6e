"""Import shim: the package lives in the directory ``no-node-comparison_amd/`` (a name Python
cannot import directly). Importing ``no_node_comparison_amd`` loads that directory as the package
of this name and replaces this shim in ``sys.modules``.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "no-node-comparison_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
