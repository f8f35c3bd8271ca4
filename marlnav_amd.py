"""Import alias: ``import marlnav_amd`` loads the package in ``marl-nav_amd/``
(a directory name that is not a Python identifier) and registers it, and its
submodules, under the importable name."""
import importlib as _importlib
import sys as _sys

_pkg = _importlib.import_module("marl-nav_amd")
for _name in ("abi", "environment", "shard", "utils"):
    _sys.modules[__name__ + "." + _name] = _sys.modules["marl-nav_amd." + _name]
_sys.modules[__name__] = _pkg
