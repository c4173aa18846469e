"""Import alias for the ``cuda-aware-mpi-on-3d-heate-quation_amd`` package.

The package directory name contains hyphens, so it cannot be imported with a
plain ``import`` statement.  ``import heat3d_amd`` loads that directory as a
package named ``heat3d_amd`` (all sub-modules resolve under this one name).
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                         "cuda-aware-mpi-on-3d-heate-quation_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
