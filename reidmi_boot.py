"""Registers the ``multimodal-reid_amd/`` directory as the importable package
``multimodal_reid_amd`` (the directory name carries a hyphen, so it cannot be
imported by name).  Entry points (bench.py, __graft_entry__.py, tests) call
``reidmi_boot.load()`` once; afterwards ``import multimodal_reid_amd.x`` works.
"""
import importlib.util
import os
import sys

PKG_NAME = "multimodal_reid_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "multimodal-reid_amd")


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod
