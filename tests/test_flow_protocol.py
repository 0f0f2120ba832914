"""CPU: a thread model of k_flow's work protocol (tests/native/flow_sim.cpp, restating
csrc/tg_flow.h's deal / lists / queue / readiness / flush rules with host atomics) runs every
chunk-step exactly once and terminates, at ragged sizes, one and several sub-problems, and run
rates from rare to every env.  The GPU suite (tests/test_gpu_flow.py) checks the kernel
itself against the per-step API and the oracle."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("flowsim") / "flow_sim")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe,
                           os.path.join(HERE, "native", "flow_sim.cpp")])
    return exe


@pytest.mark.parametrize("n,k,p,w,run", [(1, 3, 1, 4, 21), (64, 16, 8, 4, 21), (4096, 16, 8, 6, 21),
                                         (70001, 16, 2, 8, 21), (20000, 5, 3, 8, 100),
                                         (30000, 16, 4, 8, 3)])
def test_flow_protocol(sim, n, k, p, w, run):
    r = subprocess.run([sim, str(n), str(k), str(p), str(w), str(run)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
