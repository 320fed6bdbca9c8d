"""Import alias for the framework package.

The package lives in ``distributed-parameter-server-for-ml-training_amd/`` (the repository's
required layout), which is not a valid Python identifier. Importing ``psx`` loads that
directory as the package ``psx`` and replaces this module in ``sys.modules``, so
``import psx``, ``import psx.parallel.server`` and ``from psx.models import resnet`` all work
from the repository root.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "distributed-parameter-server-for-ml-training_amd")

_spec = importlib.util.spec_from_file_location(
    "psx", os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR]
)
_mod = importlib.util.module_from_spec(_spec)
sys.modules["psx"] = _mod
_spec.loader.exec_module(_mod)
