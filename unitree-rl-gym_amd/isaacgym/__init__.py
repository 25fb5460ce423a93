"""Minimal ``isaacgym`` compatibility package for the MI355X-native engine.

The reference's entry scripts start with ``import isaacgym`` and its helpers use
``gymapi.SimParams`` / ``gymutil.parse_arguments`` (legged_gym/utils/helpers.py:
49-71, 122-148).  This package provides exactly that surface (argument parsing,
sim-param containers, the torch_utils quaternion helpers) so those scripts run
unmodified.  The physics itself is ``leggedsim`` (HIP), not PhysX.
"""
