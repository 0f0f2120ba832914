"""Shared test setup.

Markers: ``gpu`` tests need an MI355X (they call the C ABI of libtg_amd.so); everything else
runs on the CPU: the oracle against the reference's golden vectors, the host-only build of
the product core against the oracle, the C-ABI library's exports, the Python surface and the
multi-process (gloo) sharding logic.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs through libtg_amd.so)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # test infrastructure: the CPU parity oracle
    O.build()
    return O


@pytest.fixture(scope="session")
def hostcheck():
    """Host-only build of the product core (tests/native)."""
    import ctypes
    d = os.path.join(ROOT, "tests", "native")
    lib = os.path.join(d, "libtg_hostcheck.so")
    subprocess.check_call(["make", "-s", "-C", d])
    L = ctypes.CDLL(lib)
    P = ctypes.c_void_p
    L.hc_run.restype = ctypes.c_int
    L.hc_run.argtypes = [P, P, P, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                         ctypes.c_uint64, ctypes.c_int, ctypes.c_int] + [P] * 8
    L.hc_set_gotab.argtypes = [ctypes.c_int]
    L.hc_predicates.restype = ctypes.c_uint
    L.hc_predicates.argtypes = [ctypes.c_int] * 3
    L.hc_predicate_table.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint, P]
    L.hc_rng_stream.restype = ctypes.c_int
    L.hc_rng_stream.argtypes = [ctypes.c_uint64, P, ctypes.c_int, ctypes.c_int, P]
    L.hc_render_run.restype = ctypes.c_int
    L.hc_render_run.argtypes = [P, P, P, ctypes.c_uint64, P, ctypes.c_int64, ctypes.c_int,
                                ctypes.c_uint64, ctypes.c_int, ctypes.c_int, P, ctypes.c_int,
                                ctypes.c_int, P]
    return L


@pytest.fixture(scope="session")
def tg():
    import gym_treasure_game_amd as tg
    return tg


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name))
