"""Host side of the drop-in boundary (CPU): gymapi value types, argument
parsing, asset import, the bit-exact env / actor / body / DOF index maps and
the tensor layouts of SURVEY.md §8a, and Isaac-Gym-style error behaviour."""
import math
import os
import sys

import numpy as np
import pytest

from isaacgym import gymapi, gymtorch, gymutil
from test_isaacgym_amd import scenes, _native as N
from conftest import ROOT, has_gpu


# ------------------------------------------------------------------ math
def test_quat_euler_roundtrip_and_rotate():
    for r, p, y in [(0.3, -0.2, 1.1), (math.pi / 2, 0, 0), (0, math.pi / 2 - 1e-3, 0.5)]:
        q = gymapi.Quat.from_euler_zyx(r, p, y)
        rr, pp, yy = q.to_euler_zyx()
        assert np.allclose([rr, pp, yy], [r, p, y], atol=1e-9)
    qx = gymapi.Quat.from_axis_angle(gymapi.Vec3(1, 0, 0), 0.5 * math.pi)   # examples/maths.py:36
    v = qx.rotate(gymapi.Vec3(0, 1, 0))
    assert np.allclose([v.x, v.y, v.z], [0, 0, 1], atol=1e-12)
    assert np.allclose(gymapi.Quat.from_euler_zyx(0.5 * math.pi, 0, 0).to_numpy(), qx.to_numpy())
    qi = qx.inverse()
    w = (qi * qx).normalize()
    assert np.allclose(w.to_numpy(), [0, 0, 0, 1])


def test_transform_compose_inverse():
    a = gymapi.Transform(gymapi.Vec3(1, 2, 3), gymapi.Quat.from_euler_zyx(0.1, 0.2, 0.3))
    b = gymapi.Transform(gymapi.Vec3(-1, 0.5, 2), gymapi.Quat.from_euler_zyx(-0.4, 0.1, 1.0))
    p = gymapi.Vec3(0.3, -0.7, 1.1)
    ab = (a * b).transform_point(p)
    ab2 = a.transform_point(b.transform_point(p))
    assert np.allclose(ab.to_numpy(), ab2.to_numpy())
    back = a.inverse().transform_point(a.transform_point(p))
    assert np.allclose(back.to_numpy(), p.to_numpy())


def test_structured_dtypes():
    assert gymapi.DofState.dtype.names == ("pos", "vel")
    rb = np.zeros(2, gymapi.RigidBodyState.dtype)
    rb["pose"]["p"]["z"] = 3.0                     # examples/projectiles.py:163-168
    assert rb["pose"]["p"]["z"][1] == 3.0
    assert set(gymapi.DOF_PROPERTIES_DTYPE.names) >= {"driveMode", "stiffness", "damping", "armature",
                                                      "hasLimits", "lower", "upper", "velocity", "effort"}


def test_parse_arguments(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["x"])
    a = gymutil.parse_arguments(description="t")
    assert a.physics_engine == gymapi.SIM_PHYSX and a.compute_device_id == 0 and a.use_gpu_pipeline
    assert a.sim_device == "cuda:0" and a.use_gpu
    monkeypatch.setattr(sys, "argv", ["x", "--num_envs", "4096", "--controller", "osc", "--pipeline", "cpu"])
    a = gymutil.parse_arguments(custom_parameters=[
        {"name": "--controller", "type": str, "default": "ik"},
        {"name": "--num_envs", "type": int, "default": 256}])   # examples/franka_cube_ik_osc.py:93-101
    assert a.num_envs == 4096 and a.controller == "osc" and not a.use_gpu_pipeline


# ------------------------------------------------------------------ assets
def test_gimbal_asset(gym):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, gymapi.SimParams())
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    a = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/gimbal.urdf", opts)
    assert gym.get_asset_rigid_body_names(a) == ["base", "yaw_link", "pitch_link", "camera_link"]
    assert gym.get_asset_dof_count(a) == 3
    assert [gym.get_asset_dof_type(a, i) for i in range(3)] == [gymapi.DOF_ROTATION] * 3
    assert gym.get_joint_type_string(gym.get_asset_joint_type(a, 0)) == "Revolute"
    p = gym.get_asset_dof_properties(a)
    assert np.all(p["hasLimits"]) and np.allclose(p["lower"], -1.57) and np.allclose(p["effort"], 10)
    assert np.allclose(p["velocity"], 1.0)
    # base link has no <inertial>: mass from its collision box at density 1000
    assert a.mass_props[0].mass == pytest.approx(1000 * 0.2 * 0.2 * 0.1)
    assert a.mass_props[1].mass == pytest.approx(0.01)
    assert np.allclose(np.diag(a.mass_props[1].inertia), 1e-4)


def test_servo_assets_and_proxies(gym):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, gymapi.SimParams())
    uav = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/uav.urdf", gymapi.AssetOptions())
    mp = uav.mass_props[0]
    assert mp.mass == 100.0 and np.allclose(mp.com, 0)
    # mass given, inertia missing: box inertia of the proxy at that mass
    assert np.allclose(np.diag(mp.inertia), [100 / 12 * (20 ** 2 + 3 ** 2), 100 / 12 * (16 ** 2 + 3 ** 2),
                                             100 / 12 * (16 ** 2 + 20 ** 2)])
    ref = "/root/reference/assets"
    if os.path.isdir(ref):   # the reference's own URDF, mesh missing -> the same frozen proxy
        r = gym.load_asset(sim, ref, "urdf/uav/urdf/rq-1-predator-mae-uav.urdf", gymapi.AssetOptions())
        assert r.bodies[0].shapes[0].size == uav.bodies[0].shapes[0].size
        assert np.allclose(r.mass_props[0].inertia, mp.inertia)
    assert gym.load_asset(sim, scenes.ASSET_ROOT, "servo/missing.urdf", gymapi.AssetOptions()) is None


# ------------------------------------------------------------------ index maps & tensors
def test_servo_index_maps_and_initial_tensors(gym):
    n = 3
    sim, envs = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    assert gym.get_sim_actor_count(sim) == 2 * n and gym.get_sim_rigid_body_count(sim) == 2 * n
    for i, env in enumerate(envs):
        assert gym.get_actor_count(env) == 2
        assert gym.get_actor_index(env, 1, gymapi.DOMAIN_SIM) == 2 * i + 1
        assert gym.get_actor_rigid_body_index(env, 1, 0, gymapi.DOMAIN_SIM) == 2 * i + 1
        assert gym.get_actor_rigid_body_index(env, 1, 0, gymapi.DOMAIN_ENV) == 1
        assert gym.get_actor_rigid_body_handle(env, 0, 0) == 0
        assert gym.find_actor_dof_handle(env, 0, "nope") == gymapi.INVALID_HANDLE
        assert gym.get_actor_name(env, 0) == "predator%d" % i
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    assert root.shape == (2 * n, 13) and rb.shape == (2 * n, 13) and dof.shape == (0, 2) and ncf.shape == (2 * n, 3)
    view = root.view(n, 2, 13)                       # test10_servo_vecenv.py:373-374
    per_row = int(math.sqrt(n))
    for i in range(n):
        ox, oy = (i % per_row) * 40.0, (i // per_row) * 40.0
        assert np.allclose(view[i, 0, :3].numpy(), [ox - 10, oy, 102])
        assert np.allclose(view[i, 1, :3].numpy(), [ox, oy, 2])
    assert np.allclose(root[:, 6].numpy(), 1.0)
    # acquire hands out one persistent storage (test10 :372 vs :400)
    assert gym.acquire_actor_root_state_tensor(sim).data_address == root.data_ptr()


def test_gimbal_dof_layout(gym):
    n = 4
    sim, envs = scenes.gimbal_scene(gym, n, use_gpu_pipeline=False)
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    assert dof.shape == (3 * n, 2)
    assert dof.view(n, 3, 2).shape == (n, 3, 2)      # test13_camera_spherical_joint.py:268 style views
    env = envs[2]
    assert gym.get_actor_dof_index(env, 0, 1, gymapi.DOMAIN_SIM) == 2 * 3 + 1
    assert gym.find_actor_rigid_body_index(env, 0, "camera_link", gymapi.DOMAIN_SIM) == 2 * 4 + 3
    props = gym.get_actor_dof_properties(env, 0)
    assert np.all(props["driveMode"] == gymapi.DOF_MODE_POS) and np.allclose(props["stiffness"], 50)
    A = sim.model_arrays
    assert A["artic_i"].shape == (n, 4) and A["artic_tmpl_i"][0].tolist() == [0, 4, 3, 1]
    assert A["tmpl_link_i"][:, 0].tolist() == [-1, 0, 1, 2]
    # link poses by forward kinematics at q = 0: joint origin 0.1 m above the base
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim)).view(n, 4, 13)
    assert np.allclose(rb[0, 1, :3].numpy() - rb[0, 0, :3].numpy(), [0, 0, 0.1], atol=1e-6)


def test_errors_are_isaac_style(gym):
    sim, envs = scenes.servo_scene(gym, 2, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    box = gym.create_box(sim, 1, 1, 1, gymapi.AssetOptions())
    assert gym.create_actor(envs[0], box, gymapi.Transform(), "late", 0, 0) == gymapi.INVALID_HANDLE
    assert gym.create_env(sim, gymapi.Vec3(), gymapi.Vec3(1, 1, 1), 1) is None
    import torch
    bad = torch.zeros((3, 13))
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(bad)) is False
    if not has_gpu():
        with pytest.raises(N.MigymError):
            gym.simulate(sim)
        ok = torch.zeros((4, 13))
        with pytest.raises(N.MigymError):
            gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(ok))


def test_indexed_setters_reject_bad_indices_and_counts(gym):
    """an indexed setter never hands the C ABI a count larger than its
    index tensor or an actor index outside [0, num_actors); Isaac Gym style, it
    returns False. (The device copy kernels also skip out-of-range rows.)"""
    import torch
    sim, envs = scenes.gimbal_scene(gym, 3, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    root = torch.zeros((3, 13))
    dofs = torch.zeros((9,))
    ds = torch.zeros((9, 2))
    for idx, count in (([0, 3], 2), ([-1], 1), ([0, 1], 3), ([0], -1)):
        it = gymtorch.unwrap_tensor(torch.tensor(idx, dtype=torch.int32))
        assert gym.set_actor_root_state_tensor_indexed(sim, gymtorch.unwrap_tensor(root), it, count) is False
        assert gym.set_dof_position_target_tensor_indexed(sim, gymtorch.unwrap_tensor(dofs), it, count) is False
        assert gym.set_dof_state_tensor_indexed(sim, gymtorch.unwrap_tensor(ds), it, count) is False
    bad_dtype = gymtorch.unwrap_tensor(torch.tensor([0], dtype=torch.int64))
    assert gym.set_dof_velocity_target_tensor_indexed(sim, gymtorch.unwrap_tensor(dofs), bad_dtype, 1) is False


def test_force_tensors_on_mixed_devices_are_rejected(gym):
    import torch
    from conftest import has_gpu
    sim, _ = scenes.servo_scene(gym, 2, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    if not has_gpu():
        with pytest.raises(N.MigymError):
            gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(torch.zeros(4, 3)), None)
        return
    f = torch.zeros(4, 3)
    t = torch.zeros(4, 3, device="cuda:0")
    assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(f), gymtorch.unwrap_tensor(t)) is False


def test_set_actor_dof_states_keeps_unselected_column(gym):
    """STATE_POS leaves velocities as they are (and STATE_VEL positions)."""
    sim, envs = scenes.gimbal_scene(gym, 2, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    st = gym.get_actor_dof_states(envs[1], 0, gymapi.STATE_ALL)
    st["pos"] = [0.1, 0.2, 0.3]
    st["vel"] = [1.0, 2.0, 3.0]
    assert gym.set_actor_dof_states(envs[1], 0, st, gymapi.STATE_ALL)
    st2 = gym.get_actor_dof_states(envs[1], 0, gymapi.STATE_ALL)
    st2["pos"] = [-0.5, -0.5, -0.5]
    st2["vel"] = [9.0, 9.0, 9.0]
    assert gym.set_actor_dof_states(envs[1], 0, st2, gymapi.STATE_POS)
    got = gym.get_actor_dof_states(envs[1], 0, gymapi.STATE_ALL)
    assert np.allclose(got["pos"], -0.5) and np.allclose(got["vel"], [1.0, 2.0, 3.0])
    st2["pos"] = [0.7, 0.7, 0.7]
    assert gym.set_actor_dof_states(envs[1], 0, st2, gymapi.STATE_VEL)
    got = gym.get_actor_dof_states(envs[1], 0, gymapi.STATE_ALL)
    assert np.allclose(got["pos"], -0.5) and np.allclose(got["vel"], 9.0)
    # env 0 untouched
    assert np.allclose(gym.get_actor_dof_states(envs[0], 0, gymapi.STATE_ALL)["vel"], 0.0)


def test_friction_parameters_scope_is_stated(gym, capsys, tmp_path):
    """physx.friction_offset_threshold / friction_correlation_distance
    (franka_cube_ik_osc.py:124-125; test10 leaves them at Isaac Gym's defaults)
    drive the friction anchors of single-shape free bodies on the ground and of
    the coupled step: no notice for such scenes. A
    free body of several collision shapes alone on the ground keeps per-point
    friction, and the first sim holding one says so on stderr."""
    from test_isaacgym_amd import _sim as S
    S._warned_multishape[0] = False
    sp = scenes.franka_sim_params(False)
    sp.physx.friction_offset_threshold = 0.0011
    sp.physx.friction_correlation_distance = 0.00051
    sim, _ = scenes.servo_scene(gym, 4, use_gpu_pipeline=False)
    sim.finalize()
    assert "per-point friction" not in capsys.readouterr().err
    urdf = tmp_path / "two_boxes.urdf"
    urdf.write_text('<robot name="two"><link name="l"><inertial><mass value="1"/>'
                    '<inertia ixx="0.1" iyy="0.1" izz="0.1" ixy="0" ixz="0" iyz="0"/></inertial>'
                    '<collision><origin xyz="0.2 0 0"/><geometry><box size="0.2 0.2 0.2"/></geometry></collision>'
                    '<collision><origin xyz="-0.2 0 0"/><geometry><box size="0.2 0.2 0.2"/></geometry></collision>'
                    '</link></robot>')
    sim2 = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim2, plane)
    asset = gym.load_asset(sim2, str(tmp_path), "two_boxes.urdf", gymapi.AssetOptions())
    env = gym.create_env(sim2, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 0.5)), "two", 0, 0)
    sim2.finalize()
    assert "free bodies with several collision shapes keep per-point friction" in capsys.readouterr().err
