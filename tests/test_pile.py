"""Known-answer tests of the free-body pile step on the oracle
(oracle/migym_oracle_pile.c, the bit-exact restatement of
test_isaacgym_amd/csrc/mg_pile.hip): coupled envs of more
than two free bodies and no articulation, built through the public gymapi as
examples/1080_balls_of_solitude.py builds them.

  - the script's pyramid of 30 balls per env falls and collapses onto the
    ground: no ball sinks into the ground or into another, and a ball at rest
    carries its own weight;
  - a vertical stack of balls and a stack of boxes stand, each body's net
    contact force equal to its weight;
  - a head-on plastic collision conserves momentum and ends with no relative
    normal velocity;
  - a box pushed below mu m g holds, above it slides at (F - mu m g) / m;
  - envs past the capacity (65 free bodies) are refused; with the script's
    --no_collisions filter the balls step as uncoupled free bodies.
Physics parity with PhysX is unpinned (PhysX is a closed binary, SURVEY.md
§8c); these pin the restatement to mechanics.
"""
import numpy as np
import pytest

from isaacgym import gymapi
from test_isaacgym_amd import scenes
import oracle
import pile_scenes as PS

G = PS.G


def _run(sim, frames, ext=None, every=None):
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    cf = None
    for k in range(frames):
        cf = oracle.step(p, m, st, dof, ext=ext)
        if every is not None:
            every(k, st, cf)
    return st, cf


def test_ball_pyramid_collapses_without_overlap(gym):
    n = 4
    sim, envs = scenes.ball_pile_scene(gym, n, use_gpu_pipeline=False)
    r, m = 0.2, 0.5

    def check(k, st, cf):
        if k % 15:
            return
        x = st[:, 0:3].reshape(n, 30, 3)
        assert x[:, :, 1].min() > r - 2e-3                        # on or above the ground (y-up)
        d = np.linalg.norm(x[:, :, None] - x[:, None], axis=-1) + 9 * np.eye(30)
        # the layers meet at ~10 m/s, 16 cm per frame against a 2 cm contact
        # offset (no speculative contacts): a transient overlap, pushed out
        # within a few frames
        tol = 4e-3 if k >= 120 else 3e-2
        assert d.min() > 2 * r - tol, "frame %d: balls overlap by %g" % (k, 2 * r - d.min())

    st, cf = _run(sim, 300, every=check)
    x = st[:, 0:3].reshape(n, 30, 3)
    assert x[:, :, 1].max() < r + 5e-3                            # the pyramid came down
    # balls resting on the ground alone carry their weight
    assert np.allclose(cf[:, 1], m * G, rtol=1e-3)


def test_vertical_ball_stack_stands(gym):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(False))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    r = 0.05
    ball = gym.create_sphere(sim, r, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    for k in range(4):
        gym.create_actor(env, ball, gymapi.Transform(gymapi.Vec3(0, 0, r + 2 * r * k + 0.002 * k)), "b%d" % k, 0, 0)
    st, cf = _run(sim, 240)
    m = 1000.0 * 4.0 / 3.0 * np.pi * r ** 3
    assert np.allclose(st[:, 2], r + 2 * r * np.arange(4), atol=2e-3)
    assert np.abs(st[:, 0:2]).max() < 1e-6                        # symmetric: no sideways drift
    assert np.allclose(cf[:, 2], m * G, rtol=2e-3)


def test_box_stack_stands(gym):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(False, npos=8, contact_offset=0.002))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    sizes = (0.3, 0.2, 0.1)
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    z = 0.0
    for k, s in enumerate(sizes):
        box = gym.create_box(sim, s, s, s, gymapi.AssetOptions())
        gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0.01 * k, -0.005 * k, z + s / 2)), "b%d" % k, 0, 0)
        z += s
    st, cf = _run(sim, 180)
    want = np.cumsum(sizes) - np.array(sizes) / 2
    assert np.allclose(st[:, 2], want, atol=3e-3)
    st2 = st.copy()
    A = sim.model_arrays
    p, m = sim.mg_params(), sim.mg_model()
    dof = A["dof_state0"].copy()
    for _ in range(60):
        cf = oracle.step(p, m, st2, dof)
    assert np.abs(st2[:, 0:3] - st[:, 0:3]).max() < 1e-3          # < 1 mm per second of creep
    mass = 1000.0 * np.array(sizes) ** 3
    assert np.allclose(cf[:, 2], mass * G, rtol=0.02)


def test_head_on_collision_conserves_momentum(gym):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(False, gravity=False))   # no ground
    r = 0.1
    ball = gym.create_sphere(sim, r, gymapi.AssetOptions())
    opts = gymapi.AssetOptions()
    opts.linear_damping = 0.0
    opts.angular_damping = 0.0
    ball = gym.create_sphere(sim, r, opts)
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    for k, x in enumerate((-1.0, 0.0, 5.0)):
        gym.create_actor(env, ball, gymapi.Transform(gymapi.Vec3(x, 0, 1)), "b%d" % k, 0, 0)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    st[0, 7] = 2.0                                                # A at 2 m/s towards B
    dof = A["dof_state0"].copy()
    for _ in range(60):
        oracle.step(p, m, st, dof)
    mass = 1000.0 * 4.0 / 3.0 * np.pi * r ** 3
    assert abs(st[0, 7] + st[1, 7] - 2.0) < 1e-5                  # momentum (equal masses)
    assert abs(st[0, 7] - st[1, 7]) < 1e-3                        # restitution 0: they move together
    assert np.abs(st[:2, 8:13]).max() < 1e-6                      # central impact: no spin, no sideways motion
    assert st[1, 0] - st[0, 0] > 2 * r - 2e-3                     # touching, not overlapping
    assert np.array_equal(st[2], A["body_state0"][2])              # the far ball never moved
    del mass


@pytest.mark.parametrize("yaw", [0.0, 0.3, 0.785])
@pytest.mark.parametrize("ratio,slides", [(0.5, False), (0.95, False), (1.05, True), (1.5, True)])
def test_box_push_below_and_above_mu_m_g(gym, ratio, slides, yaw):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(False, npos=8, contact_offset=0.002))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    plane.static_friction = plane.dynamic_friction = 1.0
    gym.add_ground(sim, plane)
    box = gym.create_box(sim, 0.2, 0.2, 0.1, gymapi.AssetOptions())
    ball = gym.create_sphere(sim, 0.05, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    pose = gymapi.Transform(gymapi.Vec3(0, 0, 0.05))
    pose.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), yaw)
    gym.create_actor(env, box, pose, "box", 0, 0)
    for k in range(2):                                            # two far balls make it a pile env
        gym.create_actor(env, ball, gymapi.Transform(gymapi.Vec3(3 + k, 3, 0.05)), "b%d" % k, 0, 0)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    mass = 1000.0 * 0.2 * 0.2 * 0.1
    mu = 0.5 * (1.0 + gym_shape_friction(A))
    for _ in range(30):
        oracle.step(p, m, st, dof)
    x0, t = st[0, 0], 60
    ext = np.zeros((3, 6), np.float32)
    ext[0, 0] = ratio * mu * mass * G
    for _ in range(t):
        oracle.step(p, m, st, dof, ext=ext)
    moved = st[0, 0] - x0
    if not slides:
        assert abs(moved) < (5e-4 if ratio < 0.6 else 2e-3), moved     # a give of < 2 mm near the limit
    else:
        T = t / 60.0
        want = 0.5 * (ratio - 1.0) * mu * G * T * T
        assert abs(moved - want) < 0.12 * want, (moved, want)


def gym_shape_friction(A):
    return float(A["shapes"][0, 11])


def test_pile_capacity_refused(gym):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(False))
    gym.add_ground(sim, gymapi.PlaneParams())
    ball = gym.create_sphere(sim, 0.02, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    for k in range(65):
        gym.create_actor(env, ball, gymapi.Transform(gymapi.Vec3(0.05 * (k % 8), 0.05 * (k // 8), 0.5)), None, 0, 0)
    with pytest.raises(RuntimeError):
        _run(sim, 1)


def test_no_collisions_mode_is_uncoupled(gym):
    """--no_collisions (group 0, filter 1): no pair may touch, so the balls are
    ordinary free bodies; they fall through each other onto the ground."""
    sim, _ = scenes.ball_pile_scene(gym, 2, use_gpu_pipeline=False, mode="none")
    st, cf = _run(sim, 240)
    assert np.allclose(st[:, 1], 0.2, atol=2e-3)                 # every ball on the ground
    assert st.shape[0] == 60


def test_mixed_pile_settles(gym, tmp_path):
    """Spheres, boxes, capsules and octahedron hulls heaped on a fixed box and
    the ground: nothing passes through the ground, and once the heaps have
    landed their kinetic energy only decays (rolling spheres keep rolling,
    slowed by the default angular damping)."""
    n = 6
    sim, info = PS.mixed_pile_scene(gym, n, False, d=str(tmp_path))
    A = sim.build_model()
    mass = 1.0 / A["body_mass"][:, 0]
    mass[~np.isfinite(mass)] = 0.0
    ke = []

    def rec(k, st, cf):
        assert np.isfinite(st).all() and np.isfinite(cf).all()
        assert st[:, 2].min() > -5e-3, k                          # nothing fell through the ground
        if k >= 90 and k % 30 == 0:
            ke.append(float((0.5 * mass * (st[:, 7:10] ** 2).sum(1)).sum()))

    _run(sim, 360, every=rec)
    assert all(b <= a * 1.001 for a, b in zip(ke, ke[1:])), ke


def test_cross_env_collisions_are_warned(gym, capsys):
    """--all_collisions (group 0, filter 0 in every env): Isaac Gym lets balls
    of different envs collide; this build steps each env on its own and says
    so once on stderr (the per-env modes stay silent)."""
    from test_isaacgym_amd import _sim
    _sim._warned_cross_env[0] = False
    for mode, warned in (("env", False), ("none", False)):
        sim, _ = scenes.ball_pile_scene(gym, 2, use_gpu_pipeline=False, mode=mode)
        _sim._warn_cross_env_contacts(sim.build_model())
        assert ("different envs" in capsys.readouterr().err) == warned
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, scenes.ball_pile_sim_params(False))
    gym.add_ground(sim, gymapi.PlaneParams())
    ball = gym.create_sphere(sim, 0.1, gymapi.AssetOptions())
    for i in range(2):
        env = gym.create_env(sim, gymapi.Vec3(-1, 0, -1), gymapi.Vec3(1, 1, 1), 2)
        for k in range(3):
            gym.create_actor(env, ball, gymapi.Transform(gymapi.Vec3(0.3 * k, 1, 0)), None, 0, 0)
    _sim._warn_cross_env_contacts(sim.build_model())
    assert "different envs" in capsys.readouterr().err


def test_cross_env_warning_group_minus_one_and_scale(capsys):
    """The warning's group rules straight on actor_coll rows (env, group,
    filter): group -1 meets every group; filter bits shared by every pair keep
    it silent; and the check is O(n log n) — test10's layout at 262,144 envs
    (group i, filter -1) takes well under a second (it took ~90 s to
    prepare_sim when the check was quadratic)."""
    import time
    from test_isaacgym_amd import _sim

    def warned(rows):
        _sim._warned_cross_env[0] = False
        _sim._warn_cross_env_contacts({"actor_coll": np.asarray(rows, dtype=np.int32)})
        return "different envs" in capsys.readouterr().err

    assert not warned([[0, 0, 0], [1, 1, 0]])                 # one env per group
    assert warned([[0, 0, 0], [1, -1, 0]])                    # group -1 joins group 0 across envs
    assert not warned([[0, 0, 1], [1, -1, 1]])                # ... but their filters share a bit
    assert warned([[0, -1, 0], [1, -1, 2]])                   # only group -1, two envs, no shared bit
    assert not warned([[0, -1, 0], [0, -1, 0]])               # only group -1, one env
    assert warned([[0, 3, 1], [0, -1, 2], [1, 3, 1]])         # group 3 spans envs; filters 1 and 2 share none
    n = 262144
    rows = np.stack([np.repeat(np.arange(n), 2), np.repeat(np.arange(n), 2), -np.ones(2 * n, np.int64)], 1)
    t0 = time.perf_counter()
    assert not warned(rows)
    assert time.perf_counter() - t0 < 2.0
