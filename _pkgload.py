"""Import helper: the package directory is named ``deeparc-sfm_amd`` (hyphenated, as the
project layout requires), so it is registered under the importable name
``deeparc_sfm_amd`` from its path."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "deeparc-sfm_amd")
NAME = "deeparc_sfm_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
