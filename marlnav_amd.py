"""Import alias: ``import marlnav_amd`` loads the package in ``marl-nav_amd/``
(a directory name that is not a Python identifier) and registers it, and its
submodules, under the importable name. ``python -m marlnav_amd`` runs the
command line (marl-nav_amd/cli.py, mirroring ``python -m marlnav``)."""
import importlib as _importlib
import sys as _sys

_pkg = _importlib.import_module("marl-nav_amd")
for _name in ("abi", "cli", "environment", "rollout", "shard", "utils"):
    _sys.modules["marlnav_amd." + _name] = _importlib.import_module("marl-nav_amd." + _name)

if __name__ == "__main__":
    _sys.exit(_sys.modules["marlnav_amd.cli"].main())
_sys.modules[__name__] = _pkg
