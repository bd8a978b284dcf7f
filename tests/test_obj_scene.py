"""Scene ingestion from XML + OBJ + bitmap files."""
import os

import numpy as np
import pytest

FLOOR_OBJ = """# floor quad with uv and normals
v -2 0 -2
v 2 0 -2
v 2 0 2
v -2 0 2
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 1 0
f 1/1/1 4/4/1 3/3/1 2/2/1
"""

BOX_OBJ = """# unit cube, quads, no normals / uvs (normals recomputed)
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
v 1 0 1
v 1 1 1
v 0 1 1
f 1 4 3 2
f 5 6 7 8
f 1 2 6 5
f 2 3 7 6
f 3 4 8 7
f 4 1 5 8
"""

XML = """<scene version="3.0.0">
  <default name="spp" value="4"/>
  <integrator type="path"><integer name="max_depth" value="8"/></integrator>
  <sensor type="perspective">
    <float name="fov" value="60"/>
    <transform name="to_world">
      <matrix value="-1 0 0 0  0 0.9701425 -0.2425356 1.5  0 -0.2425356 -0.9701425 4.0  0 0 0 1"/>
    </transform>
    <sampler type="independent"><integer name="sample_count" value="$spp"/></sampler>
    <film type="hdrfilm"><integer name="width" value="32"/><integer name="height" value="24"/><rfilter type="tent"/></film>
  </sensor>
  <bsdf type="twosided" id="FloorBSDF">
    <bsdf type="diffuse"><texture name="reflectance" type="bitmap"><string name="filename" value="checker.png"/></texture></bsdf>
  </bsdf>
  <bsdf type="twosided" id="BoxBSDF">
    <bsdf type="roughplastic"><string name="distribution" value="ggx"/><float name="alpha" value="0.2"/>
      <rgb name="diffuse_reflectance" value="0.7, 0.5, 0.3"/></bsdf>
  </bsdf>
  <shape type="obj" id="Floor_0"><string name="filename" value="floor.obj"/><ref id="FloorBSDF"/></shape>
  <shape type="obj" id="Box_0"><string name="filename" value="box.obj"/>
    <transform name="to_world"><matrix value="1 0 0 -0.5  0 1 0 0  0 0 1 -0.5  0 0 0 1"/></transform>
    <ref id="BoxBSDF"/></shape>
  <shape type="rectangle">
    <transform name="to_world"><matrix value="0.5 0 0 0  0 0 -1 2.5  0 0.5 0 0  0 0 0 1"/></transform>
    <bsdf type="twosided"><bsdf type="diffuse"><rgb name="reflectance" value="0, 0, 0"/></bsdf></bsdf>
    <emitter type="area"><rgb name="radiance" value="8, 8, 8"/></emitter>
  </shape>
</scene>
"""


@pytest.fixture(scope="module")
def scene_dir(tmp_path_factory):
    from PIL import Image

    d = tmp_path_factory.mktemp("objscene")
    (d / "floor.obj").write_text(FLOOR_OBJ)
    (d / "box.obj").write_text(BOX_OBJ)
    (d / "scene.xml").write_text(XML)
    c = (np.indices((8, 8)).sum(0) % 2).astype(np.uint8)
    img = np.stack([c * 200 + 30, c * 60 + 90, 255 - c * 200], -1).astype(np.uint8)
    Image.fromarray(img).save(d / "checker.png")
    return str(d)


def test_obj_loader_semantics(scene_dir):
    from mtx import obj

    P, N, UV, F = obj.load_obj(os.path.join(scene_dir, "floor.obj"))
    assert P.shape == (4, 3) and F.tolist() == [[0, 1, 2], [0, 2, 3]]  # fan over (1,4,3,2)
    assert np.allclose(N, [0, 1, 0])
    assert np.allclose(UV[1], [0, 0])  # vertex 4 has vt (0,1): flipped to v = 0
    P, N, UV, F = obj.load_obj(os.path.join(scene_dir, "box.obj"))
    assert P.shape == (8, 3) and F.shape == (12, 3) and UV is None
    # recomputed angle-weighted normals point away from the cube centre
    assert (np.sum(N * (P - 0.5), 1) > 0).all() and np.allclose(np.linalg.norm(N, axis=1), 1)
    _, N2, _, _ = obj.load_obj(os.path.join(scene_dir, "box.obj"), face_normals=True)
    assert N2 is None


def test_xml_scene_loads_files(scene_dir):
    from mtx import scene

    sc = scene.Scene.from_xml(os.path.join(scene_dir, "scene.xml"))
    assert sorted(sc.meta["loaded_files"]) == ["box.obj", "checker.png", "floor.obj"]
    assert sc.n_tris == 2 + 12 + 2 and sc.width == 32 and sc.height == 24
    assert sc.n_textures == 1
    tex = sc.textures[0]
    assert (tex.width, tex.height) == (8, 8)
    t = sc.texels[tex.offset:tex.offset + 3]  # texel (0, 0): sRGB (30, 90, 255), linearised
    assert np.allclose(t, [((30 / 255 + 0.055) / 1.055) ** 2.4, ((90 / 255 + 0.055) / 1.055) ** 2.4, 1.0],
                       rtol=1e-5)


def test_xml_scene_oracle_render_sane(scene_dir, oracle):
    from mtx import load_dict, scene

    sc = scene.Scene.from_xml(os.path.join(scene_dir, "scene.xml"))
    integ = load_dict({"type": "path_test"})
    f = oracle.render(sc, integ.render_args(sc, 0, 4))
    img = f[1:-1, 1:-1, :3] / f[1:-1, 1:-1, 3:]
    assert np.isfinite(img).all() and img.mean() > 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["path_test", "mypath"])
def test_xml_scene_gpu_bit_exact(scene_dir, oracle, name):
    from mtx import load_dict, scene

    sc = scene.Scene.from_xml(os.path.join(scene_dir, "scene.xml"))
    integ = load_dict({"type": name})
    film = integ.render_film(sc, seed=1, spp=4)
    np.testing.assert_array_equal(film, oracle.render(sc, integ.render_args(sc, 1, 4)))
