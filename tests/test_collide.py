"""Narrow phase of the coupled per-env step (mg_collide.h, restated by
oracle/migym_oracle_env.c:collide_) against independent float64 geometry.

Box-box: existence of contacts must agree with a float64 separating-axis test
(15 axes) outside a +-1e-4 m band around the margin; normals are unit length and
point from B towards A; every reported point lies on box A's surface shell and
within |sep| + 1e-3 m of box B. Known answers: a box resting on a larger box
(4 bottom corners, normal +z, zero separation), a sphere above a box face, an
edge-edge crossing. Parity of the device narrow phase with this restatement is
covered bit for bit by tests/test_franka_gpu.py.
"""
import math

import numpy as np

import oracle

BOX, SPHERE, CAPSULE = 1, 0, 2


def _quat(axis, ang):
    axis = np.asarray(axis, np.float64)
    axis = axis / np.linalg.norm(axis)
    s = math.sin(0.5 * ang)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, math.cos(0.5 * ang)])


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return (aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
            aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz)


def _rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _shape(t, c, q, h):
    return np.array([t, *c, *q, *h], np.float32)


def _sat(c1, R1, h1, c2, R2, h2):
    d = c2 - c1
    axes = [R1[:, i] for i in range(3)] + [R2[:, i] for i in range(3)]
    axes += [np.cross(R1[:, i], R2[:, j]) for i in range(3) for j in range(3)]
    best = -1e30
    for ax in axes:
        n = np.linalg.norm(ax)
        if n < 1e-6:
            continue
        ax = ax / n
        r1 = sum(h1[k] * abs(ax @ R1[:, k]) for k in range(3))
        r2 = sum(h2[k] * abs(ax @ R2[:, k]) for k in range(3))
        best = max(best, abs(d @ ax) - r1 - r2)
    return best


def _box_dist(p, c, R, h):
    """signed distance from p to the box surface (negative inside)."""
    loc = R.T @ (p - c)
    q = np.abs(loc) - h
    outside = np.linalg.norm(np.maximum(q, 0.0))
    return outside + min(max(q[0], q[1], q[2]), 0.0)


def test_box_box_random_against_float64_sat():
    rng = np.random.RandomState(7)
    margin = 0.01
    checked = contacts = 0
    for _ in range(3000):
        h1 = rng.uniform(0.05, 0.5, 3)
        h2 = rng.uniform(0.05, 0.5, 3)
        q1 = _quat(rng.normal(size=3), rng.uniform(-math.pi, math.pi))
        q2 = _quat(rng.normal(size=3), rng.uniform(-math.pi, math.pi))
        c1 = rng.uniform(-0.2, 0.2, 3)
        c2 = c1 + rng.normal(size=3) * rng.uniform(0.1, 1.0)
        A = _shape(BOX, c1, q1, h1)
        B = _shape(BOX, c2, q2, h2)
        # the device works in float32: compare against the float32-rounded inputs
        c1, c2 = A[1:4].astype(np.float64), B[1:4].astype(np.float64)
        R1, R2 = _rot(A[4:8].astype(np.float64)), _rot(B[4:8].astype(np.float64))
        h1, h2 = A[8:11].astype(np.float64), B[8:11].astype(np.float64)
        sep = _sat(c1, R1, h1, c2, R2, h2)
        out = oracle.collide(A, B, margin)
        if sep > margin + 1e-4:
            assert len(out) == 0, (sep, out)
        elif sep < margin - 1e-4:
            assert len(out) >= 1, sep
        checked += 1
        for p in out:
            pt, n, s = p[0:3].astype(np.float64), p[3:6].astype(np.float64), float(p[6])
            assert abs(np.linalg.norm(n) - 1.0) < 1e-5
            assert s < margin
            # the point is on A's surface shell and within |sep| of B
            assert abs(_box_dist(pt, c1, R1, h1)) < 2e-3 + abs(s), (_box_dist(pt, c1, R1, h1), s)
            assert _box_dist(pt, c2, R2, h2) < abs(s) + 2e-3
            contacts += 1
    assert checked == 3000 and contacts > 500


def test_box_resting_on_box_four_corners():
    table = _shape(BOX, (0.5, 0.0, 0.2), (0, 0, 0, 1), (0.3, 0.5, 0.2))
    for yaw in (0.0, 0.3, -1.1):
        cube = _shape(BOX, (0.45, 0.1, 0.4 + 0.0225), _quat((0, 0, 1), yaw), (0.0225, 0.0225, 0.0225))
        out = oracle.collide(cube, table, 0.001)
        assert len(out) == 4
        assert np.allclose(out[:, 3:6], [0, 0, 1], atol=1e-6)        # from the table towards the cube
        assert np.allclose(out[:, 6], 0.0, atol=1e-6)
        assert np.allclose(out[:, 2], 0.4, atol=1e-6)                # bottom face of the cube
        # the four bottom corners of the cube
        R = _rot(cube[4:8].astype(np.float64))
        corners = np.array(sorted([tuple((cube[1:4] + R @ np.array([sx, sy, -1]) * 0.0225)[:2])
                                   for sx in (-1, 1) for sy in (-1, 1)]))
        got = np.array(sorted([tuple(p[:2].astype(np.float64)) for p in out]))
        assert np.allclose(got, corners, atol=1e-5)


def test_sphere_above_box_face():
    box = _shape(BOX, (0, 0, 0), (0, 0, 0, 1), (1, 1, 1))
    sph = _shape(SPHERE, (0.2, -0.3, 1.5), (0, 0, 0, 1), (0.49, 0, 0))
    out = oracle.collide(sph, box, 0.02)
    assert len(out) == 1
    assert np.allclose(out[0, 3:6], [0, 0, 1])
    assert abs(out[0, 6] - 0.01) < 1e-6
    assert np.allclose(out[0, 0:3], [0.2, -0.3, 1.01], atol=1e-6)
    assert len(oracle.collide(sph, box, 0.005)) == 0
    # box as A: same contact seen from the other side
    out2 = oracle.collide(box, sph, 0.02)
    assert len(out2) == 1 and np.allclose(out2[0, 3:6], [0, 0, -1]) and abs(out2[0, 6] - 0.01) < 1e-6


def test_edge_edge_crossing():
    # two long thin boxes crossing at right angles, edges overlapping by 1 mm
    a = _shape(BOX, (0, 0, 0), _quat((1, 0, 0), math.pi / 4), (1.0, 0.1, 0.1))
    b = _shape(BOX, (0, 0, 2 * 0.1 * math.sqrt(2) - 0.001), _quat((0, 1, 0), math.pi / 4), (0.1, 1.0, 0.1))
    out = oracle.collide(a, b, 0.01)
    assert len(out) == 1
    n = out[0, 3:6]
    assert abs(abs(n[2]) - 1.0) < 1e-4 and n[2] < 0       # pushes a down, away from b
    assert abs(out[0, 6] + 0.001) < 1e-4


def test_capsule_caps_and_segment():
    """A capsule lying flat on a box face: its two cap contacts and the axis
    segment's (the chord clipped by the box planes, at its midpoint), all at
    zero separation with the normal +z."""
    cap = _shape(CAPSULE, (0, 0, 0.05), (0, 0, 0, 1), (0.05, 0.2, 0))
    box = _shape(BOX, (0, 0, -0.5), (0, 0, 0, 1), (1, 1, 0.5))
    out = oracle.collide(cap, box, 0.01)
    assert len(out) == 3
    assert np.allclose(out[:, 6], 0.0, atol=1e-6)
    assert np.allclose(sorted(out[:, 0]), [-0.2, 0.0, 0.2], atol=1e-6)
    assert np.allclose(out[:, 3:6], [0, 0, 1], atol=1e-6)


def test_capsule_across_narrow_box_segment_only():
    """Both caps beyond a 0.1 m wide box: no cap contact, one segment contact
    at the box's middle, penetration 1 mm (the cap spheres alone miss it)."""
    cap = _shape(CAPSULE, (0, 0, 0.049), (0, 0, 0, 1), (0.05, 0.2, 0))
    box = _shape(BOX, (0, 0, -0.5), (0, 0, 0, 1), (0.05, 1, 0.5))
    out = oracle.collide(cap, box, 0.01)
    assert len(out) == 1
    assert abs(out[0, 0]) < 1e-6 and abs(out[0, 6] + 0.001) < 1e-6
    assert np.allclose(out[0, 3:6], [0, 0, 1], atol=1e-6)


# ---------------------------------------------------------------- convex hulls
CONVEX = 3


def _hull_of_box(h):
    from test_isaacgym_amd import _assets
    pts = np.array([[sx * h[0], sy * h[1], sz * h[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
    return _assets.make_hull(pts)


def test_hull_mass_properties_match_analytic_box():
    hull = _hull_of_box((0.1, 0.2, 0.3))
    a, b, c = 0.2, 0.4, 0.6
    assert hull.volume == __import__("pytest").approx(a * b * c, rel=1e-12)
    assert np.allclose(hull.com, 0.0, atol=1e-12)
    V = a * b * c
    assert np.allclose(np.diag(hull.inertia), [V * (b * b + c * c) / 12, V * (a * a + c * c) / 12,
                                               V * (a * a + b * b) / 12], rtol=1e-9)
    assert len(hull.verts) == 8 and len(hull.planes) == 6          # coplanar triangles merged


def test_hull_of_box_matches_box_box_face_contact():
    """A box as a convex hull against a box: vertex penetration gives the same
    deepest separation and normal as the SAT / clipping box-box path for a
    face contact (random tilts of the upper box, small overlaps)."""
    rng = np.random.RandomState(3)
    h = np.array([0.05, 0.04, 0.03])
    rec = _hull_of_box(h).record()
    for _ in range(50):
        q = _quat(rng.normal(size=3), rng.uniform(-0.3, 0.3))
        R = _rot(q)
        low = np.abs(R[2, :]) @ h                                     # half height of the tilted box
        c = np.array([rng.uniform(-0.02, 0.02), rng.uniform(-0.02, 0.02), 0.2 + low - rng.uniform(0.0, 0.004)])
        B = _shape(BOX, (0, 0, 0), (0, 0, 0, 1), (0.3, 0.3, 0.2))
        A_box = _shape(BOX, c, q, h)
        A_hull = _shape(CONVEX, c, q, (float(np.linalg.norm(h)), 0, 0))
        rb = oracle.collide(A_box, B, 0.01)
        rh = oracle.collide(A_hull, B, 0.01, hull_a=rec)
        assert len(rb) and len(rh)
        assert rh[:, 6].min() == __import__("pytest").approx(rb[:, 6].min(), abs=2e-6)
        assert np.allclose(rh[np.argmin(rh[:, 6]), 3:6], [0, 0, 1], atol=1e-5)


def test_hull_edges():
    """Hull records carry their edges (vertex pairs on two common merged faces):
    a box 12, an octahedron 12, a random 32-vertex hull V + F - 2 by Euler for its
    triangulated faces (merged faces only remove diagonals)."""
    from test_isaacgym_amd import _assets
    assert len(_hull_of_box((0.1, 0.2, 0.3)).edges()) == 12
    octa = _assets.make_hull(np.array([[0.1, 0, 0], [-0.1, 0, 0], [0, 0.1, 0], [0, -0.1, 0], [0, 0, 0.1], [0, 0, -0.1]]))
    assert len(octa.edges()) == 12
    rng = np.random.RandomState(0)
    h = _assets.make_hull(rng.normal(size=(200, 3)))
    E = h.edges()
    assert len(E) == len(h.verts) + len(h.planes) - 2
    rec = h.record()
    assert rec[2] == len(E) and len(rec) == 4 + 3 * len(h.verts) + 4 * len(h.planes) + 2 * len(E)


def test_hull_edge_edge_crossing():
    """Two cube hulls turned 45 degrees about x and about y, their edges crossing
    1 mm deep with no vertex of either inside the other: found by the edge
    fallback (Cyrus-Beck chords of A's edges through B), one candidate, separation the chord
    midpoint's depth below the other cube's face (-1 mm / sqrt 2), the normal
    pushing them apart; and nothing 1 mm apart with a 0.5 mm margin."""
    h = 0.05
    rec = _hull_of_box((h, h, h)).record()
    r2 = h * math.sqrt(2)
    for depth, margin, n_expect in ((0.001, 0.01, 1), (-0.001, 0.0005, 0)):
        A = _shape(CONVEX, (0, 0, 0), _quat((1, 0, 0), math.pi / 4), (h * math.sqrt(3), 0, 0))
        B = _shape(CONVEX, (0, 0, 2 * r2 - depth), _quat((0, 1, 0), math.pi / 4), (h * math.sqrt(3), 0, 0))
        out = oracle.collide(A, B, margin, hull_a=rec, hull_b=rec)
        assert len(out) == n_expect
        for row in out:
            assert abs(row[6] + depth / math.sqrt(2)) < 2e-5
            assert row[5] < -0.7                         # normal b -> a points down
        # the box-box SAT path agrees on the crossing (one contact, depth 1 mm along z)
        if n_expect:
            Ab = _shape(BOX, A[1:4], A[4:8], (h, h, h))
            Bb = _shape(BOX, B[1:4], B[4:8], (h, h, h))
            ob = oracle.collide(Ab, Bb, margin)
            assert len(ob) == 1 and abs(ob[0, 6] + depth) < 2e-5


def test_hull_box_edge_edge_matches_sat():
    """A cube hull crossing a box edge to edge (no vertex inside): the box-edge
    branch of the edge pass gives the edge-edge normal and line distance, the
    same contact as box-box SAT (random crossing angles and depths)."""
    h = 0.05
    rec = _hull_of_box((h, h, h)).record()
    r2 = h * math.sqrt(2)
    rng = np.random.RandomState(2)
    for _ in range(20):
        depth = rng.uniform(0.0002, 0.002)
        yaw = rng.uniform(-0.5, 0.5)
        qa = _quat((1, 0, 0), math.pi / 4)
        qb = _qmul(_quat((0, 0, 1), yaw), _quat((0, 1, 0), math.pi / 4))
        for hull_on_a in (True, False):
            A = _shape(CONVEX if hull_on_a else BOX, (0, 0, 0), qa, (h * math.sqrt(3), 0, 0) if hull_on_a else (h, h, h))
            B = _shape(BOX if hull_on_a else CONVEX, (0, 0, 2 * r2 - depth), qb,
                       (h, h, h) if hull_on_a else (h * math.sqrt(3), 0, 0))
            out = oracle.collide(A, B, 0.01, hull_a=rec if hull_on_a else None, hull_b=None if hull_on_a else rec)
            ref = oracle.collide(_shape(BOX, A[1:4], A[4:8], (h, h, h)), _shape(BOX, B[1:4], B[4:8], (h, h, h)), 0.01)
            assert len(out) == 1 and len(ref) == 1
            assert abs(out[0, 6] - ref[0, 6]) < 2e-5
            assert np.allclose(out[0, 3:6], ref[0, 3:6], atol=1e-4)


def test_hull_edge_crossing_independent_of_pair_order():
    """A thin rod hull pushed through the middle of a cube hull's faces, no vertex
    of either inside the other: only the rod's edges cross the cube, the cube's
    edges miss the rod. Both pair orders find the crossing (A's edges first, then
    B's when A's find nothing), with the same separation and opposite normals."""
    rod = _hull_of_box((0.002, 0.002, 0.15)).record()
    cube = _hull_of_box((0.1, 0.1, 0.1)).record()
    q = _quat((0, 0, 1), 0.3)
    R = _shape(CONVEX, (0.01, -0.02, 0.0), q, (math.sqrt(2 * 0.002 ** 2 + 0.15 ** 2), 0, 0))
    C = _shape(CONVEX, (0, 0, 0), (0, 0, 0, 1), (0.1 * math.sqrt(3), 0, 0))
    rc = oracle.collide(R, C, 0.01, hull_a=rod, hull_b=cube)
    cr = oracle.collide(C, R, 0.01, hull_a=cube, hull_b=rod)
    assert len(rc) >= 1 and len(cr) == len(rc)
    assert np.allclose(np.sort(rc[:, 6]), np.sort(cr[:, 6]), atol=1e-6)
    assert rc[:, 6].max() < -0.05                       # deep inside the cube
    assert np.allclose(rc[np.argmin(rc[:, 6]), 3:6], -cr[np.argmin(cr[:, 6]), 3:6], atol=1e-6)


def test_hull_against_ground_and_sphere():
    from test_isaacgym_amd import _assets
    # octahedron, radius 0.1, one vertex 2 mm into a box below; a sphere resting on a face
    pts = np.array([[0.1, 0, 0], [-0.1, 0, 0], [0, 0.1, 0], [0, -0.1, 0], [0, 0, 0.1], [0, 0, -0.1]])
    hull = _assets.make_hull(pts)
    rec = hull.record()
    assert len(hull.planes) == 8
    A = _shape(CONVEX, (0, 0, 0.098), (0, 0, 0, 1), (0.1, 0, 0))
    B = _shape(BOX, (0, 0, -0.5), (0, 0, 0, 1), (1, 1, 0.5))
    r = oracle.collide(A, B, 0.001, hull_a=rec)
    assert len(r) == 1 and r[0, 6] == __import__("pytest").approx(-0.002, abs=1e-6)
    assert np.allclose(r[0, :3], [0, 0, -0.002], atol=1e-6) and np.allclose(r[0, 3:6], [0, 0, 1])
    # sphere (A) of radius 0.05 touching face (1,1,1)/sqrt3 of the octahedron (B)
    n = np.ones(3) / math.sqrt(3)
    dface = 0.1 / math.sqrt(3)
    S = _shape(SPHERE, n * (dface + 0.05 - 0.001), (0, 0, 0, 1), (0.05, 0, 0))
    r = oracle.collide(S, _shape(CONVEX, (0, 0, 0), (0, 0, 0, 1), (0.1, 0, 0)), 0.01, hull_b=rec)
    assert len(r) == 1 and r[0, 6] == __import__("pytest").approx(-0.001, abs=1e-6)
    assert np.allclose(r[0, 3:6], n, atol=1e-6)


def test_reference_franka_meshes_become_hulls():
    import os
    from isaacgym import gymapi
    from conftest import REFERENCE
    from test_isaacgym_amd import _assets
    root = os.path.join(REFERENCE, "assets")
    if not os.path.isdir(root):
        __import__("pytest").skip("reference tree not present")
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    a = _assets.load_urdf(root, "urdf/franka_description/robots/franka_panda.urdf", opts)
    shapes = [s for b in a.bodies for s in b.shapes]
    assert all(s.type == _assets.CONVEX for s in shapes) and len(shapes) == 11
    assert all(4 <= len(s.hull.verts) <= 32 and len(s.hull.planes) <= 64 for s in shapes)
    # mass from the hulls at density 1000 (no <inertial> in the URDF)
    assert a.mass_props[1].mass == __import__("pytest").approx(1000 * shapes[1].hull.volume, rel=1e-9)


def test_obb_screen_never_drops_a_contact():
    """The coupled step's OBB pair screen (mg_env.hip obb_apart, DESIGN.md §3.6
    step 2) against the narrow phase it guards: over random poses of a random
    hull against a box and against another hull, near contact, every pair the
    screen rejects yields no contact from the full test (it only removes work),
    and it does reject the pairs that are clearly apart along a face axis."""
    from test_isaacgym_amd import _assets
    rng = np.random.RandomState(7)
    hull = _assets.make_hull(rng.normal(size=(60, 3)) * np.array([0.08, 0.02, 0.03]))
    rec = hull.record()
    rad = float(np.max(np.linalg.norm(hull.verts, axis=1)))
    hb = (0.05, 0.05, 0.05)
    rejected = kept_empty = 0
    for k in range(3000):
        qa = rng.normal(size=4)
        qb = rng.normal(size=4)
        qa /= np.linalg.norm(qa)
        qb /= np.linalg.norm(qb)
        d = rng.normal(size=3)
        d *= rng.uniform(0.0, 0.25) / np.linalg.norm(d)
        A = _shape(CONVEX, (0.0, 0.0, 0.0), tuple(qa), (rad, 0, 0))
        if k % 2:
            B = _shape(1, tuple(d), tuple(qb), hb)
            out = oracle.collide(A, B, 0.01, hull_a=rec)
            apart = oracle.obb_apart(A, B, 0.01, hull_a=rec)
        else:
            B = _shape(CONVEX, tuple(d), tuple(qb), (rad, 0, 0))
            out = oracle.collide(A, B, 0.01, hull_a=rec, hull_b=rec)
            apart = oracle.obb_apart(A, B, 0.01, hull_a=rec, hull_b=rec)
        if apart:
            rejected += 1
            assert len(out) == 0, (k, out)
        elif len(out) == 0:
            kept_empty += 1
    assert rejected > 500          # the screen removes a good share of the near-miss pairs
