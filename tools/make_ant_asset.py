"""Writes assets/mjcf/ant.xml: the physics content of the reference's
assets/mjcf/nv_ant.xml (compiler, defaults, the body / joint / geom tree,
motor actuators) re-serialized without rendering-only elements (textures,
materials, lights, colours), so the GPU box, which has no /root/reference, can
load the same ant (examples/apply_forces.py:67). Run in this container:
    python tools/make_ant_asset.py [/root/reference/assets/mjcf/nv_ant.xml]
"""
import os
import sys
import xml.etree.ElementTree as ET

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/assets/mjcf/nv_ant.xml"
DST = os.path.join(ROOT, "assets", "mjcf", "ant.xml")
KEEP_ATTR = {"rgba", "material", "texture", "condim", "margin"}


def strip(el):
    out = ET.Element(el.tag, {k: v for k, v in el.attrib.items() if k not in KEEP_ATTR})
    for c in el:
        if c.tag in ("light", "camera", "site"):
            continue
        out.append(strip(c))
    return out


def main():
    src = ET.parse(SRC).getroot()
    dst = ET.Element("mujoco", {"model": src.get("model", "ant")})
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
    main()
