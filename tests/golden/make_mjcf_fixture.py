"""Raw MJCF attribute fixture for the compiled-model tests (tests/test_model_tables.py).

Test infrastructure, run in the build container where /root/reference exists:

    python tests/golden/make_mjcf_fixture.py [REFERENCE_ROOT]

It reads the reference's two model files as plain XML (no MuJoCo, and deliberately NOT
tools/compile_model.py, so the fixture is an independent reading of the MJCF) and writes the
attribute values the physics depends on to tests/golden/mjcf_raw.json: body frames and
inertials, joint types/axes/ranges/armature/damping with the default classes applied, actuator
gains/biases/ranges, the tendon, the equality, the keyframe, option, contact exclusions and the
colliding-geom parameters of the cubes, pads and scene boxes.

Sources: mujoco_manip/data/franka_emika_panda/panda.xml:6-36 (defaults), :120-250 (bodies),
:253-285 (tendon/equality/actuators/exclude); mujoco_manip/data/pick_and_place_scene.xml:4
(option), :40-125 (scene geoms, bins, cubes), :130-135 (keyframe).
"""
from __future__ import annotations

import json
import os
import sys
import xml.etree.ElementTree as ET

HERE = os.path.dirname(os.path.abspath(__file__))


def floats(s, n=None, default=None):
    if s is None:
        return default
    v = [float(x) for x in s.split()]
    if n is not None and len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


class Defaults:
    """Nested <default class=...> tables: class -> tag -> attributes (inherited)."""

    def __init__(self, root):
        self.table = {}
        top = root.find("default")
        if top is not None:
            self._walk(top, "main", {})

    def _walk(self, node, cls, inherited):
        own = {tag: dict(attrs) for tag, attrs in inherited.items()}
        for ch in node:
            if ch.tag != "default":
                own.setdefault(ch.tag, {}).update(ch.attrib)
        self.table[cls] = own
        for ch in node:
            if ch.tag == "default":
                self._walk(ch, ch.attrib["class"], own)

    def attrs(self, cls, tag, el):
        out = dict(self.table.get(cls, {}).get(tag, {}))
        out.update(el.attrib)
        return out


def walk_bodies(node, defaults, cls, out, parent):
    for b in node.findall("body"):
        bcls = b.attrib.get("childclass", cls)
        rec = {
            "parent": parent,
            "pos": floats(b.attrib.get("pos"), 3, [0.0, 0.0, 0.0]),
            "quat": floats(b.attrib.get("quat"), 4, [1.0, 0.0, 0.0, 0.0]),
            "joints": [],
            "geoms": [],
        }
        inert = b.find("inertial")
        if inert is not None:
            rec["mass"] = float(inert.attrib["mass"])
            rec["ipos"] = floats(inert.attrib.get("pos"), 3, [0.0, 0.0, 0.0])
            if "fullinertia" in inert.attrib:
                rec["fullinertia"] = floats(inert.attrib["fullinertia"], 6)
            else:
                rec["diaginertia"] = floats(inert.attrib["diaginertia"], 3)
        for j in b.findall("joint"):
            a = defaults.attrs(j.attrib.get("class", bcls), "joint", j)
            rec["joints"].append({
                "name": a["name"], "type": a.get("type", "hinge"),
                "axis": floats(a.get("axis"), 3, [0.0, 0.0, 1.0]),
                "range": floats(a.get("range"), 2),
                "armature": float(a.get("armature", 0.0)), "damping": float(a.get("damping", 0.0)),
            })
        for j in b.findall("freejoint"):
            rec["joints"].append({"name": j.attrib["name"], "type": "free"})
        for g in b.findall("geom"):
            a = defaults.attrs(g.attrib.get("class", bcls), "geom", g)
            if a.get("contype", "1") == "0" and a.get("conaffinity", "1") == "0":
                continue  # visual only
            rec["geoms"].append({
                "name": a.get("name"), "type": a.get("type", "sphere"), "mesh": a.get("mesh"),
                "size": floats(a.get("size")), "pos": floats(a.get("pos"), 3, [0.0, 0.0, 0.0]),
                "mass": float(a["mass"]) if "mass" in a else None,
                "condim": int(a.get("condim", 3)), "friction": floats(a.get("friction"), None, [1.0, 0.005, 0.0001]),
            })
        out[b.attrib["name"]] = rec
        walk_bodies(b, defaults, bcls, out, b.attrib["name"])


def main(ref_root):
    data = os.path.join(ref_root, "mujoco_manip", "data")
    panda = ET.parse(os.path.join(data, "franka_emika_panda", "panda.xml")).getroot()
    scene = ET.parse(os.path.join(data, "pick_and_place_scene.xml")).getroot()
    dp = Defaults(panda)

    bodies = {}
    walk_bodies(panda.find("worldbody"), dp, "main", bodies, "world")
    walk_bodies(scene.find("worldbody"), Defaults(scene), "main", bodies, "world")
    world_geoms = []
    for g in scene.find("worldbody").findall("geom"):
        world_geoms.append({"name": g.attrib.get("name"), "type": g.attrib.get("type"),
                            "size": floats(g.attrib.get("size"))})

    actuators = []
    for a in panda.find("actuator"):
        at = dp.attrs(a.attrib.get("class", "main"), "general", a)
        gain = floats(at.get("gainprm"), None, [1.0])
        bias = floats(at.get("biasprm"), None, [0.0, 0.0, 0.0]) + [0.0, 0.0, 0.0]
        actuators.append({
            "name": at["name"], "joint": at.get("joint"), "tendon": at.get("tendon"),
            "gain": gain[0], "bias": bias[:3], "biastype": at.get("biastype"),
            "ctrlrange": floats(at.get("ctrlrange"), 2), "forcerange": floats(at.get("forcerange"), 2),
        })

    ten = panda.find("tendon").find("fixed")
    tendon = {"name": ten.attrib["name"],
              "joints": [[j.attrib["joint"], float(j.attrib["coef"])] for j in ten.findall("joint")]}
    eq = panda.find("equality").find("joint")
    equality = {"joint1": eq.attrib["joint1"], "joint2": eq.attrib["joint2"],
                "solref": floats(eq.attrib["solref"]), "solimp": floats(eq.attrib["solimp"])}
    exclude = [[e.attrib["body1"], e.attrib["body2"]] for e in panda.find("contact").findall("exclude")]
    key = [k for k in scene.find("keyframe") if k.attrib.get("name") == "scene_start"][0]
    opt = scene.find("option").attrib
    option = {"timestep": float(opt["timestep"]), "gravity": floats(opt["gravity"], 3),
              "integrator": panda.find("option").attrib.get("integrator")}

    fixture = {
        "_source": "tests/golden/make_mjcf_fixture.py over the reference MJCF (panda.xml, pick_and_place_scene.xml)",
        "bodies": bodies, "world_geoms": world_geoms, "actuators": actuators, "tendon": tendon,
        "equality": equality, "exclude": exclude,
        "key_qpos": floats(key.attrib["qpos"]), "key_ctrl": floats(key.attrib["ctrl"]), "option": option,
    }
    out = os.path.join(HERE, "mjcf_raw.json")
    with open(out, "w") as f:
        json.dump(fixture, f, indent=1, sort_keys=True)
    print("wrote", out, len(bodies), "bodies")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
