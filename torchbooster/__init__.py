"""``import torchbooster`` compatibility namespace.

Scripts written against yliess86/TorchBooster (``import torchbooster.config``,
``torchbooster.utils.step``, ``torchbooster.distributed.launch`` ...) run
unchanged: every public reference module name resolves to its MI355X-native
implementation in :mod:`torchbooster_amd`.
"""
import importlib as _importlib
import sys as _sys

import torchbooster_amd as _impl

_MODULES = ("config", "distributed", "utils", "scheduler", "callbacks", "metrics", "dataset", "lmdb")

for _name in _MODULES:
    _mod = _importlib.import_module(f"torchbooster_amd.{_name}")
    _sys.modules[f"{__name__}.{_name}"] = _mod
    globals()[_name] = _mod

__version__ = _impl.__version__
__all__ = list(_MODULES)
