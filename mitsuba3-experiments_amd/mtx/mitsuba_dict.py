"""Scene dictionaries of ``mi.load_dict`` -> the mtx scene description.

The reference scripts build their scenes as Mitsuba dictionaries --
``mi.load_dict(mi.cornell_box())`` at path.py:308-309, path-mis.py:162,
restirgi.py:595-599 and nrc.py:130-136 -- and hand the loaded ``mi.Scene`` to
``mi.render``. :func:`spec_from_dict` converts such a dictionary (plain Python
values plus ``to_world`` transforms that expose a 4x4 ``.matrix``, as
``mi.ScalarTransform4f`` does) into the spec that
:meth:`mtx.scene.Scene.bedroom` builds from (the structure
:func:`mtx.xmlscene.parse_scene_xml` returns for an XML file), and
:func:`scene_from_dict` builds the :class:`mtx.scene.Scene`.
:func:`mtx.integrators.register_with_mitsuba` routes ``mi.load_dict`` /
``mi.load_file`` through them, so a registered mtx integrator renders the
``mi.Scene`` a script loaded.

Supported (the reference scripts' subset): a ``perspective`` sensor (fov,
fov_axis x / y / smaller / larger, near / far clip, ``hdrfilm`` size) with
a ``to_world`` transform; BSDFs diffuse, roughplastic, conductor,
roughconductor, dielectric, roughdielectric, twosided, mask, with rgb /
scalar / bitmap values and ``ref`` references; shapes rectangle, cube and
obj (``filename``, read from ``base_dir``), with an ``area`` emitter on
rectangles; a ``constant`` environment emitter (``radiance`` rgb or float;
mtx_core/interaction.h). Anything else -- including an ``obj`` whose file is
missing and ``envmap`` environments (see ENV_EMITTERS) -- raises
:class:`mtx.MtxError` rather than rendering a different scene.
"""
from __future__ import annotations

import numpy as np

from ._lib import MtxError

BSDF_TYPES = {"diffuse", "roughplastic", "conductor", "roughconductor", "dielectric", "roughdielectric",
              "twosided", "mask"}
SHAPE_TYPES = {"rectangle", "cube", "obj"}
SENSOR_TYPES = {"perspective"}
_IGNORED = {"integrator", "sampler"}  # scene entries that do not describe geometry or appearance
# Environment emitters: the reference integrators read them where a ray
# escapes (path-mis.py:41 valid_ray = scene.environment() is not None;
# path.py:239 / path-mis.py:84 si.emitter(scene).eval on a miss) and NEE picks
# them among the scene's emitters. mtx evaluates a ``constant`` one (uniform
# radiance, uniform sphere sampling); an ``envmap`` (a bitmap over the sphere
# with its own importance sampling) is refused.
ENV_EMITTERS = {"constant", "envmap"}
OTHER_EMITTERS = {"point", "spot", "directional", "projector", "directionalarea"}


def _matrix(t):
    if t is None:
        return None
    m = getattr(t, "matrix", t)
    a = np.asarray(m, dtype=np.float64)
    if a.shape != (4, 4):
        raise MtxError(f"to_world: expected a 4x4 transform, got shape {a.shape}")
    return [float(x) for x in a.reshape(-1)]


def _value(v):
    """rgb / spectrum / scalar / bitmap property -> the spec's form."""
    if isinstance(v, dict):
        t = v.get("type")
        if t in ("rgb", "spectrum"):
            val = v.get("value")
            val = [float(val)] * 3 if np.isscalar(val) else [float(x) for x in val]
            return val
        if t == "bitmap":
            return {k: (_value(x) if isinstance(x, dict) else x) for k, x in v.items()}
        raise MtxError(f"unsupported texture / value type {t!r}")
    if isinstance(v, (list, tuple, np.ndarray)):
        return [float(x) for x in v]
    if hasattr(v, "__len__") and not isinstance(v, str):  # Dr.Jit / mitsuba colour types
        return [float(x) for x in v]
    return v


def _bsdf(d: dict, key: str | None = None) -> dict:
    t = d.get("type")
    if t not in BSDF_TYPES:
        raise MtxError(f"unsupported bsdf type {t!r}")
    out = {"type": t}
    if key is not None:
        out["id"] = key
    nested = [(k, v) for k, v in d.items() if isinstance(v, dict) and v.get("type") in BSDF_TYPES]
    if t in ("twosided", "mask"):
        if len(nested) != 1:
            raise MtxError(f"{t}: expected exactly one nested bsdf, got {len(nested)}")
        out["nested"] = _bsdf(nested[0][1])
    if t in ("conductor", "roughconductor") and d.get("material", "none") != "none":
        raise MtxError(f"{t}: named conductor materials ({d['material']!r}) are not supported; give eta / k")
    for k, v in d.items():
        if k in ("type", "id") or (isinstance(v, dict) and v.get("type") in BSDF_TYPES):
            continue
        if t == "mask" and k == "opacity":
            val = _value(v)
            out["opacity"] = float(val[0] if isinstance(val, list) else val)
            continue
        out[k] = _value(v)
    return out


def _sensor(d: dict) -> dict:
    film = d.get("film", {}) or {}
    rf = film.get("rfilter")
    return {"type": d["type"], "fov": float(d.get("fov", 45.0)), "fov_axis": d.get("fov_axis", "x"),
            "near_clip": float(d.get("near_clip", 1e-2)), "far_clip": float(d.get("far_clip", 1e4)),
            "to_world": _matrix(d.get("to_world")) or [float(x) for x in np.eye(4).reshape(-1)],
            "film": {"type": film.get("type", "hdrfilm"), "width": int(film.get("width", 768)),
                     "height": int(film.get("height", 576)),
                     "rfilter": (rf.get("type") if isinstance(rf, dict) else getattr(rf, "type", None)) or "gaussian"}}


def spec_from_dict(d: dict) -> dict:
    """A ``mi.load_dict`` scene dictionary -> the mtx scene spec."""
    if d.get("type") != "scene":
        raise MtxError(f"expected a scene dictionary (type 'scene'), got {d.get('type')!r}")
    sensor, bsdfs, shapes, env = None, {}, [], None
    for key, v in d.items():
        if key == "type" or not isinstance(v, dict):
            continue
        t = v.get("type")
        if t in SENSOR_TYPES:
            if sensor is not None:
                raise MtxError("more than one sensor")
            sensor = _sensor(v)
        elif t in BSDF_TYPES:
            bsdfs[key] = _bsdf(v, key)
        elif t in SHAPE_TYPES:
            sd = {"id": key, "type": t, "to_world": _matrix(v.get("to_world"))}
            for k, x in v.items():
                if k in ("type", "to_world", "bsdf", "emitter"):
                    continue
                sd[k] = _value(x)
            b = v.get("bsdf")
            if b is None:
                sd["bsdf_inline"] = {"type": "diffuse", "reflectance": [0.5, 0.5, 0.5]}  # Mitsuba's default BSDF
            elif not isinstance(b, dict):
                raise MtxError(f"shape {key!r}: bsdf must be a dictionary")
            elif b.get("type") == "ref":
                sd["bsdf"] = b["id"]
            else:
                sd["bsdf_inline"] = _bsdf(b)
            em = v.get("emitter")
            if t == "obj" and not v.get("filename"):
                raise MtxError(f"shape {key!r}: an obj shape needs a filename")
            if em is not None:
                if em.get("type") != "area" or t != "rectangle":
                    raise MtxError(f"shape {key!r}: only area emitters on rectangles are supported")
                sd["emitter"] = {"type": "area", "radiance": _value(em.get("radiance", [1.0, 1.0, 1.0]))}
            shapes.append(sd)
        elif t in _IGNORED or key in _IGNORED:
            continue
        elif t == "constant":
            if env is not None:
                raise MtxError("more than one environment emitter")
            env = {"type": "constant", "radiance": _value(v.get("radiance", 1.0))}
        elif t in ENV_EMITTERS:
            raise MtxError(f"scene entry {key!r}: environment emitter {t!r} is not supported -- mtx evaluates "
                           "rectangle area emitters and a constant environment only "
                           "(path-mis.py:41 / :84 would read the envmap where a ray escapes)")
        elif t in OTHER_EMITTERS:
            raise MtxError(f"scene entry {key!r}: {t!r} emitters are not supported (rectangle area emitters only)")
        else:
            raise MtxError(f"scene entry {key!r}: unsupported type {t!r}")
    if sensor is None:
        raise MtxError("the scene has no perspective sensor")
    if env is None and not any("emitter" in s for s in shapes):
        raise MtxError("the scene has no emitter")
    for s in shapes:
        if "bsdf" in s and s["bsdf"] not in bsdfs:
            raise MtxError(f"shape {s['id']!r} references the unknown bsdf {s['bsdf']!r}")
    spec = {"defaults": {}, "integrator": d.get("integrator"), "sensor": sensor, "bsdfs": bsdfs, "shapes": shapes}
    if env is not None:
        spec["environment"] = env
    return spec


def scene_from_dict(d: dict, base_dir: str | None = None, tex_res: int = 512):
    """mi.load_dict(d) for the supported subset -> :class:`mtx.scene.Scene`.
    Mesh and bitmap files are read from `base_dir` (default: the working
    directory, as mi.load_dict resolves them); a missing one raises."""
    return scene_from_spec(spec_from_dict(d), base_dir, tex_res)


def scene_from_spec(spec: dict, base_dir: str | None = None, tex_res: int = 512):
    """A converted spec (:func:`spec_from_dict`) -> :class:`mtx.scene.Scene`."""
    import os

    from .scene import Scene

    return Scene.bedroom(spec=spec, base_dir=base_dir or os.getcwd(), tex_res=tex_res, strict=True)


def sensor_from_dict(d: dict) -> dict:
    """A ``perspective`` sensor dictionary (the ``sensor`` argument of
    mi.render / SamplingIntegrator.render) -> the spec's sensor form."""
    if not isinstance(d, dict) or d.get("type") not in SENSOR_TYPES:
        raise MtxError(f"unsupported sensor {d.get('type') if isinstance(d, dict) else type(d).__name__!r} "
                       "(perspective only)")
    return _sensor(d)
