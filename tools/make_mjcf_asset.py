"""Writes assets/mjcf/<name>.xml: the physics content of one of the
reference's MJCF assets (compiler, defaults, the body / joint / geom tree,
motor actuators) re-serialized without rendering-only elements (textures,
materials, lights, cameras, sites, colours), so the GPU box, which has no
/root/reference, can load the same model:
    assets/mjcf/ant.xml       <- nv_ant.xml      (examples/apply_forces.py:67)
    assets/mjcf/humanoid.xml  <- nv_humanoid.xml (examples/joint_monkey.py:35)
Run in this container:
    python tools/make_mjcf_asset.py            (both)
    python tools/make_mjcf_asset.py SRC.xml DST_NAME
"""
import os
import sys
import xml.etree.ElementTree as ET

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/assets/mjcf"
JOBS = [(os.path.join(REF, "nv_ant.xml"), "ant"), (os.path.join(REF, "nv_humanoid.xml"), "humanoid")]
KEEP_ATTR = {"rgba", "material", "texture", "condim", "margin"}


def strip(el):
    out = ET.Element(el.tag, {k: v for k, v in el.attrib.items() if k not in KEEP_ATTR})
    for c in el:
        if c.tag in ("light", "camera", "site"):
            continue
        out.append(strip(c))
    return out


def convert(SRC, name):
    DST = os.path.join(ROOT, "assets", "mjcf", name + ".xml")
    src = ET.parse(SRC).getroot()
    dst = ET.Element("mujoco", {"model": src.get("model", name)})
    for tag in ("compiler", "default", "worldbody", "actuator"):
        el = src.find(tag)
        if el is None:
            continue
        el = strip(el)
        if tag == "worldbody":          # world geoms (the floor) are not part of the asset
            for g in el.findall("geom"):
                el.remove(g)
        dst.append(el)
    ET.indent(dst)
    os.makedirs(os.path.dirname(DST), exist_ok=True)
    ET.ElementTree(dst).write(DST)
    print("wrote", DST)


if __name__ == "__main__":
    for src, name in ([(sys.argv[1], sys.argv[2])] if len(sys.argv) > 2 else JOBS):
        convert(src, name)
