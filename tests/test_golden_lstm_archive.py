"""The recurrent-policy fixtures are the reference's archives' weights (oracle/check_lstm_fixtures.py):
every parameter of tests/golden/lstm_policy_<robot>.npz equals, byte for byte, the raw tensor storage
of deploy/pre_train/<robot>/motion.pt (read from the zip, nothing unpickled or executed), and the
memory states are those of the fixture's own 5-step post-reset run.  Needs /root/reference (the
build container); skipped where it is absent (the GPU box)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "deploy", "pre_train")), reason="reference absent")
@pytest.mark.parametrize("robot", ["g1", "h1", "h1_2"])
def test_lstm_fixture_is_the_archive(robot):
    import check_lstm_fixtures as chk
    assert chk.check(REF, robot) == []
