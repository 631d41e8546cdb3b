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
