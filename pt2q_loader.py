"""Import helper: the package directory `snlp---tenary-post-train-quantization_amd/` is not a
Python identifier, so it is loaded by path and registered as module `pt2q`.

    import pt2q_loader; pt2q = pt2q_loader.load()
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "snlp---tenary-post-train-quantization_amd")
NAME = "pt2q"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[NAME]
        raise
    return mod
