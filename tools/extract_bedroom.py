"""Derive the committed bedroom description from the reference scene file.

Reads data/bedroom/scene.xml of the reference checkout (Mitsuba XML, data
only) and writes mitsuba3-experiments_amd/mtx/data/bedroom.json: sensor,
film, the 31 BSDF declarations, the 72 shapes with their transforms,
face_normals flags, emitters and the Git-LFS byte sizes of the (absent) OBJ
meshes, from which the proxy's per-shape triangle budgets are derived
(SURVEY.md §8d). Run in the build container, where the reference is
present; the GPU box only reads the JSON.

    python tools/extract_bedroom.py [/root/reference/data/bedroom/scene.xml]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mitsuba3-experiments_amd"))

from mtx.xmlscene import parse_scene_xml  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/bedroom/scene.xml"
    scene = parse_scene_xml(src)
    scene["source"] = "reference data/bedroom/scene.xml (Mitsuba XML 3.0.0)"
    out = os.path.join(HERE, "..", "mitsuba3-experiments_amd", "mtx", "data", "bedroom.json")
    with open(out, "w") as f:
        json.dump(scene, f, indent=1, sort_keys=True)
    n_obj = sum(1 for s in scene["shapes"] if s["type"] == "obj")
    print(f"wrote {out}: {len(scene['bsdfs'])} bsdfs, {len(scene['shapes'])} shapes ({n_obj} obj)")


if __name__ == "__main__":
    main()
