"""gym.apply_rigid_body_force_at_pos_tensors (examples/apply_forces_at_pos.py:126):
a force at a point is the force at the centre of mass plus the torque
(p - c) x F for the next simulate. Two sims of free boxes (no gravity, one box
per env, a centre of mass off the box origin): one gets forces at points, the
other the equivalent force + torque through apply_rigid_body_force_tensors
(computed in float64 here); their states agree, and LOCAL_SPACE with the
identity orientation equals ENV_SPACE at the shifted point."""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _sim(gym, n):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, 0)
    sp.dt, sp.substeps = 1.0 / 60.0, 2
    sp.use_gpu_pipeline = True
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    box = gym.create_box(sim, 0.4, 0.2, 0.1, gymapi.AssetOptions())
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 2), 8)
        h = gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0, 0, 1)), "box", i, -1)
        props = gym.get_actor_rigid_body_properties(env, h)
        props[0].com = gymapi.Vec3(0.05, -0.02, 0.01)
        gym.set_actor_rigid_body_properties(env, h, props)
    gym.prepare_sim(sim)
    return sim


def test_force_at_pos_equals_force_plus_torque(gym):
    n = 16
    a, b = _sim(gym, n), _sim(gym, n)
    rng = np.random.RandomState(3)
    F = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    off = rng.uniform(-0.2, 0.2, (n, 3)).astype(np.float32)
    rba = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(a))
    rbb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(b))
    for k in range(3):
        gym.refresh_rigid_body_state_tensor(a)
        gym.refresh_rigid_body_state_tensor(b)
        st = rbb.cpu().numpy().astype(np.float64)
        P = rba[:, 0:3].clone() + torch.from_numpy(off).to(DEV)
        assert gym.apply_rigid_body_force_at_pos_tensors(a, gymtorch.unwrap_tensor(torch.from_numpy(F).to(DEV)),
                                                         gymtorch.unwrap_tensor(P.contiguous()), gymapi.ENV_SPACE)
        # b: the same wrench by hand (float64): torque about the centre of mass
        q = st[:, 3:7]
        com = np.array([0.05, -0.02, 0.01])
        u, w = q[:, 0:3], q[:, 3:4]
        t = 2.0 * np.cross(u, com)
        c = st[:, 0:3] + com + w * t + np.cross(u, t)
        tau = np.cross(st[:, 0:3] + off - c, F).astype(np.float32)
        assert gym.apply_rigid_body_force_tensors(b, gymtorch.unwrap_tensor(torch.from_numpy(F).to(DEV)),
                                                  gymtorch.unwrap_tensor(torch.from_numpy(tau).to(DEV)),
                                                  gymapi.ENV_SPACE)
        gym.simulate(a)
        gym.simulate(b)
    gym.refresh_rigid_body_state_tensor(a)
    gym.refresh_rigid_body_state_tensor(b)
    ga, gb = rba.cpu().numpy(), rbb.cpu().numpy()
    assert np.abs(gb[:, 10:13]).max() > 0.1                   # it spins
    assert np.allclose(ga, gb, rtol=1e-4, atol=1e-5), np.abs(ga - gb).max()


def test_force_at_pos_local_space(gym):
    """LOCAL_SPACE at rest with the identity orientation: force and point in
    the body frame equal ENV_SPACE with the point moved to the body's position."""
    n = 4
    a, b = _sim(gym, n), _sim(gym, n)
    rba = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(a))
    rbb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(b))
    gym.refresh_rigid_body_state_tensor(a)
    F = torch.tensor([[0.0, 0.0, 30.0]] * n, device=DEV)
    pl = torch.tensor([[0.2, 0.1, 0.0]] * n, device=DEV)
    assert gym.apply_rigid_body_force_at_pos_tensors(a, gymtorch.unwrap_tensor(F), gymtorch.unwrap_tensor(pl),
                                                     gymapi.LOCAL_SPACE)
    pw = (rba[:, 0:3] + pl).contiguous()
    assert gym.apply_rigid_body_force_at_pos_tensors(b, gymtorch.unwrap_tensor(F), gymtorch.unwrap_tensor(pw),
                                                     gymapi.ENV_SPACE)
    gym.simulate(a)
    gym.simulate(b)
    gym.refresh_rigid_body_state_tensor(a)
    gym.refresh_rigid_body_state_tensor(b)
    assert np.abs(rba.cpu().numpy()[:, 10:13]).max() > 0.1
    assert np.array_equal(rba.cpu().numpy(), rbb.cpu().numpy())
