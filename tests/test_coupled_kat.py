"""Known-answer tests of the coupled per-env step (oracle/migym_oracle_env.c,
the bit-exact restatement of test_isaacgym_amd/csrc/mg_env.hip) on scenes built
through the public gymapi, as a user of examples/franka_cube_ik_osc.py would:

  - a cube at rest on a fixed table (group i, filter 0): it stays on the table
    top, the net contact force carries its weight;
  - two free boxes stacked on the ground (free-free rows): the stack stands,
    each box's net contact force equals its own weight;
  - a cube dropped on the table comes to rest on it;
  - an arm joint driven against its limit by a large effort stays at the limit
    (joint limits are unilateral solver rows).
"""
import numpy as np
import pytest

from isaacgym import gymapi
from test_isaacgym_amd import scenes
import oracle

G = 9.8


def _sim(gym, npos=8, dt=1.0 / 60.0, contact_offset=0.001):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, -G)
    sp.dt = dt
    sp.substeps = 2
    sp.use_gpu_pipeline = False
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = npos
    sp.physx.num_velocity_iterations = 1
    sp.physx.contact_offset = contact_offset
    sp.physx.rest_offset = 0.0
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    return sim


def _run(sim, frames, tgt=None):
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    if tgt is None:
        tgt = np.zeros((max(len(dof), 1), 3), np.float32)
        tgt[:len(dof), 0] = dof[:, 0]
    cf = None
    for _ in range(frames):
        cf = oracle.step(p, m, st, dof, tgt=tgt, props=A["dof_props"] if len(dof) else None)
    return st, dof, cf


def _run_more(sim, st, frames):
    A = sim.model_arrays
    p, m = sim.mg_params(), sim.mg_model()
    st = st.copy()
    dof = A["dof_state0"].copy()
    cf = None
    for _ in range(frames):
        cf = oracle.step(p, m, st, dof)
    return st, dof, cf


def test_cube_rests_on_table(gym):
    sim = _sim(gym)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    table = gym.create_box(sim, 0.6, 1.0, 0.4, opts)
    cube = gym.create_box(sim, 0.05, 0.05, 0.05, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, table, gymapi.Transform(gymapi.Vec3(0.5, 0, 0.2)), "table", 0, 0)
    pose = gymapi.Transform(gymapi.Vec3(0.45, 0.1, 0.4 + 0.025))
    pose.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), 0.4)
    gym.create_actor(env, cube, pose, "cube", 0, 0)
    st, _, cf = _run(sim, 120)
    mass = 1000.0 * 0.05 ** 3
    assert abs(st[1, 2] - 0.425) < 1e-4
    assert np.linalg.norm(st[1, 0:2] - [0.45, 0.1]) < 1e-3
    # Gauss-Seidel over the 4 corner rows leaves a small bounded wobble
    assert np.linalg.norm(st[1, 7:10]) < 2e-3 and np.linalg.norm(st[1, 10:13]) < 0.05
    assert abs(cf[1, 2] - mass * G) < 0.01 * mass * G and np.linalg.norm(cf[1, :2]) < 1e-3


def test_free_box_stack(gym):
    sim = _sim(gym)
    big = gym.create_box(sim, 0.2, 0.2, 0.2, gymapi.AssetOptions())
    small = gym.create_box(sim, 0.1, 0.1, 0.1, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, big, gymapi.Transform(gymapi.Vec3(0, 0, 0.1)), "big", 0, 0)
    gym.create_actor(env, small, gymapi.Transform(gymapi.Vec3(0.02, -0.01, 0.25)), "small", 0, 0)
    st, _, cf = _run(sim, 180)
    m1, m2 = 1000.0 * 0.2 ** 3, 1000.0 * 0.1 ** 3
    assert abs(st[0, 2] - 0.1) < 2e-3 and abs(st[1, 2] - 0.25) < 3e-3
    # positions are static; the reported velocity keeps the single velocity
    # iteration's Gauss-Seidel residual (constant, not integrated)
    assert np.linalg.norm(st[:, 7:10]) < 5e-3 and np.linalg.norm(st[:, 10:13]) < 0.05
    p0 = st[:, 0:7].copy()
    st2, _, _ = _run_more(sim, st, 60)
    assert np.abs(st2[:, 0:7] - p0).max() < 5e-4       # < 0.5 mm per second of creep
    # ground pushes (m1 + m2) g up on the big box, the small box pushes m2 g down
    assert abs(cf[0, 2] - m1 * G) < 0.02 * (m1 + m2) * G
    assert abs(cf[1, 2] - m2 * G) < 0.02 * m2 * G


def test_cube_dropped_on_table_settles(gym):
    sim = _sim(gym)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    table = gym.create_box(sim, 0.6, 1.0, 0.4, opts)
    cube = gym.create_box(sim, 0.05, 0.05, 0.05, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, table, gymapi.Transform(gymapi.Vec3(0.5, 0, 0.2)), "table", 0, 0)
    pose = gymapi.Transform(gymapi.Vec3(0.5, 0.0, 0.7))
    pose.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(1, 1, 0), 0.5)
    gym.create_actor(env, cube, pose, "cube", 0, 0)
    st, _, _ = _run(sim, 240)
    assert abs(st[1, 2] - 0.425) < 2e-3          # on a face, on the table
    assert np.linalg.norm(st[1, 7:10]) < 5e-3 and np.linalg.norm(st[1, 10:13]) < 0.05
    assert 0.2 < st[1, 0] < 0.8 and -0.5 < st[1, 1] < 0.5


def test_franka_joint_held_at_limit(gym):
    """Arm joint 4 (limits -3.0718..-0.0698) pushed towards its upper limit with
    the full 87 N m effort for 1 s: it stops at the limit."""
    sim, info = scenes.franka_scene(gym, 1, use_gpu_pipeline=False)
    A = sim.build_model()
    props = A["dof_props"].copy()
    lo, hi = props[3, 5], props[3, 6]
    # the other arm joints hold their pose (position drives), so the reaction of
    # joint 4's effort does not swing the arm into the table
    for j in (0, 1, 2, 4, 5, 6):
        props[j, 0], props[j, 1], props[j, 2] = 1.0, 400.0, 40.0
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    dof[3, 0] = hi - 0.05
    tgt = np.zeros((9, 3), np.float32)
    tgt[:, 0] = dof[:, 0]
    tgt[3, 2] = 87.0
    qmax = -1e9
    for _ in range(60):
        oracle.step(p, m, st, dof, tgt=tgt, props=props)
        qmax = max(qmax, float(dof[3, 0]))
    assert qmax <= hi + 2e-3
    assert abs(dof[3, 0] - hi) < 5e-3
    assert abs(dof[3, 1]) < 0.05
    assert np.all(np.isfinite(st))


def _cube_on_table(gym, corr=None):
    sim = _sim(gym)
    if corr is not None:
        sim.params.physx.friction_correlation_distance = corr
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    table = gym.create_box(sim, 0.6, 1.0, 0.4, opts)
    # a flat tile (10 x 10 x 2 cm, 0.2 kg): a sideways push at its centre tips
    # it only above 5 m g, so it slides rather than tips at mu m g = m g
    cube = gym.create_box(sim, 0.1, 0.1, 0.02, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, table, gymapi.Transform(gymapi.Vec3(0.5, 0, 0.2)), "table", 0, 0)
    gym.create_actor(env, cube, gymapi.Transform(gymapi.Vec3(0.45, 0.1, 0.41)), "tile", 0, 0)
    A = sim.build_model()
    return sim, A, sim.mg_params(), sim.mg_model()


def _patch(fc, pair=None):
    """(anchor count, held, record floats) of an env-0 pair in an oracle cache
    (default: the one pair holding a patch — the cube on the table)"""
    fc = fc.env
    if pair is None:
        held = [i for i in range(128) if fc[0, i * 17 + 16] != 0.0]
        assert len(held) == 1, held
        pair = held[0]
    r = fc[0, pair * 17:(pair + 1) * 17]
    return int(r[0]), r[16] != 0.0, r


@pytest.mark.parametrize("push", [0.5, 0.8, 1.2])
def test_friction_anchor_holds_or_slides(gym, push):
    """DESIGN.md §3.6.1 (patch friction): a tile (m g = 1.96 N, mu = 1) on the
    table pushed sideways by a constant force. Below mu m g the friction
    anchors hold it: after a sub-0.3 mm give in the first steps it does not
    move at all, the patch's two anchors kept step after step, bit for bit;
    above it the patch slips (anchors dropped and regrown) and the cube
    accelerates at (F - mu m g) / m."""
    sim, A, p, m = _cube_on_table(gym)
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    fc = oracle.contact_cache(m)
    mass = 1000.0 * 0.1 * 0.1 * 0.02
    for _ in range(30):   # settle
        oracle.step(p, m, st, dof, contact_cache=fc)
    cnt, held, _ = _patch(fc)
    assert cnt == 2 and held
    ext = np.zeros((2, 6), np.float32)
    F = push * mass * G
    ext[1, 0] = F
    x0 = float(st[1, 0])
    frames = 120 if push < 1.0 else 30
    xs, recs = [], []
    for _ in range(frames):
        oracle.step(p, m, st, dof, ext=ext, contact_cache=fc)
        xs.append(float(st[1, 0]))
        recs.append(_patch(fc))
    if push < 1.0:
        assert abs(xs[-1] - x0) < 3e-4
        assert abs(xs[-1] - xs[60]) < 2e-5
        assert all(c == 2 and h for c, h, _ in recs[60:])
        assert np.array_equal(recs[-1][2], recs[60][2])      # the same anchors, bit for bit
    else:
        t = frames / 60.0
        d_expect = 0.5 * (F - mass * G) / mass * t * t
        assert abs((xs[-1] - x0) - d_expect) < 0.1 * d_expect
        assert abs(st[1, 2] - 0.41) < 1e-3                  # slides flat on the table


def test_friction_anchor_spacing(gym):
    """The second anchor is the first contact farther than the correlation
    distance from the first; with a correlation distance above the cube's
    diagonal a single anchor carries the patch (and the whole Coulomb bound),
    and the tile still rests."""
    for corr, want in ((0.025, 2), (0.3, 1)):
        sim, A, p, m = _cube_on_table(gym, corr)
        st = A["body_state0"].copy()
        dof = A["dof_state0"].copy()
        fc = oracle.contact_cache(m)
        for _ in range(60):
            oracle.step(p, m, st, dof, contact_cache=fc)
        cnt, held, r = _patch(fc)
        assert held and cnt == want, (corr, cnt)
        if cnt == 2:
            assert np.linalg.norm(r[4:7] - r[10:13]) > corr
        assert abs(st[1, 2] - 0.41) < 1e-4 and np.linalg.norm(st[1, 0:2] - [0.45, 0.1]) < 1e-4


def test_friction_anchor_teleport_reanchors(gym):
    """a caller that teleports a body needs no reset of the
    friction patches — an anchor whose two copies end up farther apart than the
    correlation distance is dropped. A resting tile moved 5 cm sideways in the
    state (set_actor_root_state's effect) keeps its new place: its patch is
    re-anchored there instead of pulling it back towards the old anchors."""
    sim, A, p, m = _cube_on_table(gym)
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    fc = oracle.contact_cache(m)
    for _ in range(30):
        oracle.step(p, m, st, dof, contact_cache=fc)
    _, _, before = _patch(fc)
    before = before.copy()
    st[1, 0] += 0.05
    x1 = float(st[1, 0])
    for _ in range(30):
        oracle.step(p, m, st, dof, contact_cache=fc)
    cnt, held, after = _patch(fc)
    assert cnt == 2 and held
    assert not np.allclose(after[7:10], before[7:10])     # B-side (table) copies moved with the tile
    assert abs(float(st[1, 0]) - x1) < 1e-4                # not pulled back 5 cm
    assert np.linalg.norm(st[1, 7:10]) < 5e-3
