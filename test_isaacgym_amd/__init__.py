"""test_isaacgym_amd — MI355X-native rigid-body engine behind the Isaac Gym
tensor API (gymapi / gymtorch / gymutil / torch_utils).

The `isaacgym` package at the repository root re-exports these modules so the
reference's scripts import them unmodified (`from isaacgym import gymapi`).
"""
from . import _native  # noqa: F401  (loads libmigym.so; raises if it is missing)

__version__ = "0.1.0"
