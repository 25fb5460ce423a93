"""Runs one of the build's entry scripts (``legged_gym/scripts/<name>``) unmodified, as
``__main__`` with the given command line, for ``tests/test_gpu_scripts.py``.  Test
infrastructure only: ``play.py`` sets ``cfg.env.test``, which paces the roll-out to real
time (legged_robot.py:631-635: 10 episodes = 200 s of wall clock), so ``time.sleep`` is
replaced by a virtual sleep: it advances ``time.perf_counter`` (the pacing's clock) by the
requested time instead of waiting, and the total is printed at exit."""
import atexit
import os
import runpy
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "unitree-rl-gym_amd")
sys.path.insert(0, PKG)

_slept = [0.0, 0]


def _sleep(s):
    _slept[0] += s
    _slept[1] += 1


_perf_counter = time.perf_counter
time.sleep = _sleep
time.perf_counter = lambda: _perf_counter() + _slept[0]
atexit.register(lambda: print(f"script_runner: paced sleep requested {_slept[0]:.3f} s in {_slept[1]} calls"))
script = os.path.join(PKG, "legged_gym", "scripts", sys.argv[1])
sys.argv = [script] + sys.argv[2:]
runpy.run_path(script, run_name="__main__")
