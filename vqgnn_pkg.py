"""Import helper: the package directory is ``vq-gnn_amd/`` (hyphenated, as the
project layout requires), which Python cannot import by name; ``load()``
registers it as the package ``vq_gnn_amd`` so ``import vq_gnn_amd.vq`` works."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "vq-gnn_amd")


def load():
    mod = sys.modules.get("vq_gnn_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "vq_gnn_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vq_gnn_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
