"""Importer pieces of SURVEY.md §8(f) rank 2 on the host: COLLADA (.dae)
collision meshes (assets/urdf/anymal_b_simple_description's meshes are .dae),
reduced to convex hulls like OBJ / STL."""
import os
import textwrap

import numpy as np
import pytest

from isaacgym import gymapi
from test_isaacgym_amd import _assets
from conftest import REFERENCE

# a unit cube (8 vertices) placed by a node transform: scale 2, then translate (1, 0, 0);
# <unit meter="0.5"> halves everything
DAE = textwrap.dedent("""\
    <?xml version="1.0" encoding="utf-8"?>
    <COLLADA xmlns="http://www.collada.org/2005/11/COLLADASchema" version="1.4.1">
      <asset><unit name="half" meter="0.5"/><up_axis>Z_UP</up_axis></asset>
      <library_geometries>
        <geometry id="cube-mesh" name="cube">
          <mesh>
            <source id="cube-pos">
              <float_array id="cube-pos-array" count="24">0 0 0 1 0 0 0 1 0 1 1 0 0 0 1 1 0 1 0 1 1 1 1 1</float_array>
            </source>
            <vertices id="cube-verts"><input semantic="POSITION" source="#cube-pos"/></vertices>
            <triangles count="0"><input semantic="VERTEX" source="#cube-verts" offset="0"/><p></p></triangles>
          </mesh>
        </geometry>
      </library_geometries>
      <library_visual_scenes>
        <visual_scene id="Scene">
          <node id="outer"><translate>1 0 0</translate>
            <node id="inner"><scale>2 2 2</scale><instance_geometry url="#cube-mesh"/></node>
          </node>
        </visual_scene>
      </library_visual_scenes>
    </COLLADA>
""")


def test_collada_vertices_units_and_node_transforms(tmp_path):
    p = tmp_path / "cube.dae"
    p.write_text(DAE)
    v = _assets._mesh_vertices(str(p))
    assert v.shape == (8, 3)
    # (x * 2 + 1, y * 2, z * 2) * 0.5
    assert np.allclose(v.min(0), [0.5, 0.0, 0.0]) and np.allclose(v.max(0), [1.5, 1.0, 1.0])


def test_urdf_with_dae_collision_mesh_becomes_a_hull(gym, tmp_path):
    (tmp_path / "cube.dae").write_text(DAE)
    (tmp_path / "m.urdf").write_text(textwrap.dedent("""\
        <robot name="m"><link name="l">
          <collision><geometry><mesh filename="cube.dae" scale="0.1 0.1 0.1"/></geometry></collision>
          <inertial><mass value="1"/><inertia ixx="0.01" iyy="0.01" izz="0.01" ixy="0" ixz="0" iyz="0"/></inertial>
        </link></robot>"""))
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, gymapi.SimParams())
    a = gym.load_asset(sim, str(tmp_path), "m.urdf", gymapi.AssetOptions())
    sh = a.bodies[0].shapes
    assert len(sh) == 1 and sh[0].type == _assets.CONVEX and sh[0].source == "mesh-hull:cube.dae"
    ext = sh[0].hull.verts.max(0) - sh[0].hull.verts.min(0)
    assert np.allclose(ext, [0.1, 0.1, 0.1], atol=1e-6)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "assets")), reason="reference tree absent")
def test_reference_anymal_dae_meshes():
    """The anymal meshes of the reference (Blender COLLADA, millimetres scaled by
    the URDF's 0.001): the DAE vertices span the same box as the OBJ exports of
    the same meshes (those are y-up: obj (x, y, z) = dae (x, z, -y))."""
    d = os.path.join(REFERENCE, "assets/urdf/anymal_b_simple_description/meshes")
    for name in ("anymal_foot", "anymal_hip_l", "anymal_thigh_l", "anymal_shank_r"):
        v = _assets._mesh_vertices(os.path.join(d, name + ".dae"))
        o = _assets._mesh_vertices(os.path.join(d, name + ".obj"))
        o_zup = np.stack([o[:, 0], -o[:, 2], o[:, 1]], 1)
        assert len(v) > 1000
        assert np.allclose(v.min(0), o_zup.min(0), atol=1.5) and np.allclose(v.max(0), o_zup.max(0), atol=1.5)


def _u_obj(path, depth=1.0):
    """A U-shaped prism (two posts on a bar, 3 x 3 x depth, volume 7 depth) as a
    closed OBJ triangle mesh."""
    poly = [(0, 0), (3, 0), (3, 3), (2, 3), (2, 1), (1, 1), (1, 3), (0, 3)]
    n = len(poly)
    lines = ["v %g %g %g" % (x - 1.5, y - 1.5, z - 0.5 * depth) for z in (0.0, depth) for (x, y) in poly]
    for i in range(n):
        j = (i + 1) % n
        lines += ["f %d %d %d" % (i + 1, j + 1, n + j + 1), "f %d %d %d" % (i + 1, n + j + 1, n + i + 1)]
    for t in [[0, 1, 4], [0, 4, 5], [1, 2, 3], [1, 3, 4], [0, 5, 6], [0, 6, 7]]:
        lines.append("f %d %d %d" % (t[2] + 1, t[1] + 1, t[0] + 1))
        lines.append("f %d %d %d" % (n + t[0] + 1, n + t[1] + 1, n + t[2] + 1))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def _u_urdf(d, scale=0.1):
    _u_obj(os.path.join(d, "u.obj"))
    with open(os.path.join(d, "u.urdf"), "w") as f:
        f.write(textwrap.dedent("""\
            <robot name="u"><link name="u">
              <inertial><mass value="1"/><inertia ixx="0.01" iyy="0.01" izz="0.01" ixy="0" ixz="0" iyz="0"/></inertial>
              <collision><geometry><mesh filename="u.obj" scale="%g %g %g"/></geometry></collision>
            </link></robot>""" % (scale, scale, scale)))
    return "u.urdf"


def test_convex_decomposition_of_a_concave_mesh(gym, tmp_path):
    """AssetOptions.vhacd_enabled (examples/convex_decomposition.py's option): a
    U-shaped mesh becomes several convex hulls that keep its gap empty and
    whose volumes sum to the solid's (the single hull fills the gap)."""
    from scipy.spatial import ConvexHull
    d = str(tmp_path)
    f = _u_urdf(d)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, gymapi.SimParams())
    one = gym.load_asset(sim, d, f, gymapi.AssetOptions())
    opts = gymapi.AssetOptions()
    opts.vhacd_enabled = True
    opts.vhacd_params.max_convex_hulls = 8
    dec = gym.load_asset(sim, d, f, opts)
    s1, sd = one.bodies[0].shapes, dec.bodies[0].shapes
    assert len(s1) == 1 and 2 <= len(sd) <= 8
    assert all(s.type == _assets.CONVEX for s in sd)
    vol = 0.0
    gap = np.array([0.0, 0.05, 0.0])           # the middle of the U's gap (scale 0.1)
    for s in sd:
        v = s.hull.verts @ _assets._qmat(s.q).T + s.p
        h = ConvexHull(v)
        vol += h.volume
        assert np.any(h.equations @ np.append(gap, 1.0) > 1e-9), "a piece covers the gap"
    assert abs(vol - 7e-3) < 0.15 * 7e-3, vol
    assert ConvexHull(s1[0].hull.verts).volume > 8.5e-3        # the single hull: 9e-3, gap included


def test_mjcf_include_and_unmodelled_elements(gym, tmp_path, capsys):
    """MJCF <include file=.../> (open_ai_assets/hand/shadow_hand.xml:8-15): the
    included file's top-level children replace the include, recursively and
    relative to the including file; tendons / equality constraints, which this
    build does not model, are said on stderr rather than dropped silently."""
    sub = tmp_path / "parts"
    sub.mkdir()
    (sub / "robot.xml").write_text(textwrap.dedent('''\
        <mujoco>
          <body name="base" pos="0 0 1">
            <geom type="box" size="0.1 0.1 0.1"/>
            <include file="arm.xml"/>
          </body>
        </mujoco>'''))
    (sub / "arm.xml").write_text(textwrap.dedent('''\
        <mujoco>
          <body name="arm" pos="0 0 0.3">
            <joint name="j0" type="hinge" axis="0 1 0" range="-45 45"/>
            <geom type="capsule" fromto="0 0 0 0 0 0.2" size="0.03"/>
          </body>
        </mujoco>'''))
    (tmp_path / "top.xml").write_text(textwrap.dedent('''\
        <mujoco model="inc">
          <worldbody><include file="parts/robot.xml"/></worldbody>
          <tendon><fixed name="t"><joint joint="j0" coef="1"/></fixed></tendon>
        </mujoco>'''))
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, gymapi.SimParams())
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    a = gym.load_asset(sim, str(tmp_path), "top.xml", opts)
    assert a is not None
    assert gym.get_asset_rigid_body_names(a) == ["base", "arm"]
    assert gym.get_asset_dof_names(a) == ["j0"]
    assert "1 tendons not modelled" in capsys.readouterr().err
