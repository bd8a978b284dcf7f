"""Mitsuba 3 XML subset reader (scene ingestion for the bedroom scene).

Covers what ``data/bedroom/scene.xml`` uses: ``<default>``
and ``$name`` substitution (scene.xml:2-9), the perspective sensor with its
``to_world`` matrix, ``hdrfilm`` and ``tent`` rfilter (:10-25), BSDF
declarations with nested ``twosided`` / ``mask`` (:26-219), ``<ref>``, ``obj``
and ``rectangle`` shapes with ``to_world`` and ``face_normals`` (:221-738) and
area emitters (:706-731). The result is a plain-dict description; geometry
files are referenced, not loaded (the bedroom meshes are Git-LFS pointers and
are replaced by the deterministic proxy in :mod:`mtx.proxy`).
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

__all__ = ["parse_scene_xml", "lfs_pointer_size"]


def _subst(value: str, defaults: dict) -> str:
    if value.startswith("$") and value[1:] in defaults:
        return defaults[value[1:]]
    return value


def _floats(s: str) -> list[float]:
    return [float(x) for x in s.replace(",", " ").split()]


def _props(el, defaults) -> dict:
    """Leaf properties of a plugin element (float/integer/rgb/string/boolean)."""
    out = {}
    for c in el:
        name = c.get("name")
        if name is None:
            continue
        val = c.get("value")
        if val is not None:
            val = _subst(val, defaults)
        if c.tag == "float":
            out[name] = float(val)
        elif c.tag == "integer":
            out[name] = int(val)
        elif c.tag == "boolean":
            out[name] = val.lower() == "true"
        elif c.tag == "string":
            out[name] = val
        elif c.tag == "rgb":
            out[name] = _floats(val)
        elif c.tag == "texture":
            tex = {"type": c.get("type")}
            tex.update(_props(c, defaults))
            out[name] = tex
    return out


def _matrix(el) -> list[float] | None:
    tr = el.find("transform[@name='to_world']")
    if tr is None:
        return None
    m = tr.find("matrix")
    if m is None:
        return None
    vals = _floats(m.get("value"))
    assert len(vals) == 16, "only 4x4 <matrix> transforms are supported"
    return vals


def _bsdf(el, defaults) -> dict:
    d = {"type": el.get("type")}
    if el.get("id"):
        d["id"] = el.get("id")
    d.update(_props(el, defaults))
    nested = el.find("bsdf")
    if nested is not None:
        d["nested"] = _bsdf(nested, defaults)
    return d


def lfs_pointer_size(path: str) -> int | None:
    """Byte size recorded in a Git-LFS pointer file, or None if not a pointer."""
    try:
        with open(path, "rb") as f:
            head = f.read(512)
    except OSError:
        return None
    if not head.startswith(b"version https://git-lfs"):
        return None
    for line in head.decode("ascii", "replace").splitlines():
        if line.startswith("size "):
            return int(line.split()[1])
    return None


def parse_scene_xml(path: str, overrides: dict | None = None) -> dict:
    root = ET.parse(path).getroot()
    base = os.path.dirname(os.path.abspath(path))
    defaults = {d.get("name"): d.get("value") for d in root.findall("default")}
    defaults.update({k: str(v) for k, v in (overrides or {}).items()})

    integ = root.find("integrator")
    integrator = {"type": _subst(integ.get("type"), defaults)} if integ is not None else None
    if integ is not None:
        integrator.update(_props(integ, defaults))

    sen = root.find("sensor")
    film_el = sen.find("film")
    rf = film_el.find("rfilter")
    sampler = sen.find("sampler")
    sensor = {
        "type": sen.get("type"),
        **_props(sen, defaults),
        "to_world": _matrix(sen),
        "film": {"type": film_el.get("type"), **_props(film_el, defaults),
                 "rfilter": rf.get("type") if rf is not None else "gaussian"},
        "sampler": {"type": sampler.get("type"), **_props(sampler, defaults)} if sampler is not None else None,
    }

    bsdfs = {}
    for b in root.findall("bsdf"):
        bd = _bsdf(b, defaults)
        bsdfs[bd["id"]] = bd

    shapes = []
    for s in root.findall("shape"):
        sd = {"id": s.get("id"), "type": s.get("type"), **_props(s, defaults)}
        sd["to_world"] = _matrix(s)
        ref = s.find("ref")
        inline = s.find("bsdf")
        if ref is not None:
            sd["bsdf"] = ref.get("id")
        elif inline is not None:
            sd["bsdf_inline"] = _bsdf(inline, defaults)
        em = s.find("emitter")
        if em is not None:
            sd["emitter"] = {"type": em.get("type"), **_props(em, defaults)}
        fn = sd.get("filename")
        if fn:
            sd["lfs_size"] = lfs_pointer_size(os.path.join(base, fn))
        shapes.append(sd)
    spec = {"defaults": defaults, "integrator": integrator, "sensor": sensor, "bsdfs": bsdfs, "shapes": shapes}
    envs = root.findall("emitter")  # top-level emitters: environments
    for e in envs:
        t = _subst(e.get("type"), defaults)
        if t != "constant" or len(envs) > 1:
            from ._lib import MtxError
            raise MtxError(f"{path}: top-level emitter {t!r}: only one constant environment is supported")
        spec["environment"] = {"type": "constant", "radiance": _props(e, defaults).get("radiance", 1.0)}
    return spec
