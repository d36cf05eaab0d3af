# Before any test module imports torch (also in spawned rank processes, which
# import this package first): see tests/torch_loader_check.py.
from tests.torch_loader_check import ensure_torch_loadable as _ensure

_ensure()
