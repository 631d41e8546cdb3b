"""Drop-in import path for the reference's scripts: `from isaacgym import gymapi`
(test10_servo_vecenv.py:7-9, examples/franka_cube_ik_osc.py:16-19) resolves to
the MI355X-native implementation in test_isaacgym_amd."""
import sys as _sys

from test_isaacgym_amd import gymapi, gymtorch, gymutil, torch_utils  # noqa: F401

for _name, _mod in (("gymapi", gymapi), ("gymtorch", gymtorch), ("gymutil", gymutil),
                    ("torch_utils", torch_utils)):
    _sys.modules["isaacgym." + _name] = _mod
