"""Import alias for the package directory ``quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd``.

The directory name required by the build layout contains a hyphen, which Python cannot
import directly; this module loads it as the package ``tneq_qc_amd`` (submodules resolve
through its ``__path__``), so ``import tneq_qc_amd.contractor`` etc. work everywhere.
"""
import importlib.util
import os
import sys

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                     "quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_ROOT, "__init__.py"), submodule_search_locations=[_ROOT])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
