"""Test helper: the product kernel body compiled for the host (libsfl_hostsim.so)."""
import importlib
import os

pkg_build = importlib.import_module("network-distributed-q-learning_amd.build")
_lib = importlib.import_module("network-distributed-q-learning_amd._lib")

_cache = {}


def lib():
    if "lib" not in _cache:
        path = pkg_build.build_hostsim()
        _cache["lib"] = _lib.Lib(path)
        _cache["lib"].check_fresh()
    return _cache["lib"]
