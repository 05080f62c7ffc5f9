"""Import shim: exposes the package directory `crosscoder-model-diff-replication_amd/`
(a name that is not a Python identifier) as the module `crosscoder_amd`."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "crosscoder-model-diff-replication_amd")
_spec = importlib.util.spec_from_file_location("crosscoder_amd", os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["crosscoder_amd"] = _mod
_spec.loader.exec_module(_mod)
