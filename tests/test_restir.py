"""ReSTIR GI (restirgi.py:151-588): HIP frames vs the CPU restatement.

Every frame's film and the persistent state (samples, temporal / spatial
reservoirs, search radii) must match the oracle bit for bit (per-pixel
tolerance 0: both sides run the same IEEE operation sequence, see
test_gpu_parity.py). Configurations cover the property switches of
restirgi.py:157-166 and a camera that moves between frames
(test-restir-dynamic.py), which exercises the reprojection of
temporal_resampling (:370-380).
"""
import ctypes as C

import numpy as np
import pytest

CONFIGS = {
    # test-restir-spatial.py "biased" / "unbiased" settings
    "biased": {"jacobian": False, "bias_correction": False, "max_M_spatial": 500, "max_M_temporal": 30},
    "unbiased": {"jacobian": False, "bias_correction": True, "max_M_spatial": 500, "max_M_temporal": 30},
    # reference defaults except max_M_spatial (None raises at :297 upstream)
    "defaults": {"max_M_spatial": 500},
    "hemisphere_ss": {"bsdf_sampling": False, "spatial_spatial_reuse": True, "max_M_spatial": 40,
                      "jacobian": True, "bias_correction": False, "initial_search_radius": 6.0},
}


def _oracle_frames(oracle, scene, props, frames, cameras=None, spp=1):
    from mtx import load_dict

    integ = load_dict({"type": "restirgi", **props})
    orc = oracle.RestirOracle(scene, spp)
    out = []
    for fr in range(frames):
        if cameras is not None:
            scene.camera = cameras[fr]
        integ.n = fr
        out.append(orc.frame(scene, integ.render_args(scene, fr, spp)))
    return out, orc


def test_restir_oracle_invariants(small_scene, oracle):
    """Reservoir bookkeeping of the restatement: M after frame 0 is 1 (one
    initial sample, the zero reservoir merged), M clamps hold, W >= 0 and
    finite, radii stay in [minimal, initial]."""
    sc = small_scene.with_film(24, 16)
    props = dict(CONFIGS["biased"])
    films, orc = _oracle_frames(oracle, sc, props, 1)
    M_t = orc.tres[5, :, 2].view(np.uint32)
    assert (M_t == 1).all()
    films, orc = _oracle_frames(oracle, sc, props, 4)
    M_t = orc.tres[5, :, 2].view(np.uint32)
    M_s = orc.sres[5, :, 2].view(np.uint32)
    assert M_t.max() <= 30 and M_s.max() <= 500 and M_t.min() >= 1
    for res in (orc.tres, orc.sres):
        W = res[5, :, 1]
        assert np.isfinite(W).all() and (W >= 0).all()
    assert (orc.radius >= 3.0).all() and (orc.radius <= 10.0).all()
    for f in films:
        assert np.isfinite(f).all()
        # splats sit on pixel corners (integer positions): pixels 0..W-2 receive
        # four of weight 1/4, the last row / column two
        assert np.allclose(f[1:-2, 1:-2, 3], 1.0)
    # deterministic
    films2, _ = _oracle_frames(oracle, sc, props, 4)
    assert all(np.array_equal(a, b) for a, b in zip(films, films2))


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_restir_frames_bit_exact(small_scene, oracle, cfg):
    from mtx import load_dict

    sc = small_scene.with_film(40, 24)
    props = CONFIGS[cfg]
    frames = 4
    ref, orc = _oracle_frames(oracle, sc, props, frames)
    integ = load_dict({"type": "restirgi", **props})
    for fr in range(frames):
        film = integ.render_film(sc, seed=fr, spp=1)
        np.testing.assert_array_equal(film, ref[fr], err_msg=f"frame {fr}")
    np.testing.assert_array_equal(integ.state("sample"), orc.cur)
    np.testing.assert_array_equal(integ.state("temporal"), orc.tres)
    np.testing.assert_array_equal(integ.state("spatial"), orc.sres)
    np.testing.assert_array_equal(integ.state("radius"), orc.radius)
    assert ref[-1][..., :3].sum() > 0


@pytest.mark.gpu
def test_restir_two_samples_per_pixel_bit_exact(small_scene, oracle):
    """spp = 2 lanes per pixel (to_idx's sample_offset, restirgi.py:173)."""
    from mtx import load_dict

    sc = small_scene.with_film(24, 16)
    ref, orc = _oracle_frames(oracle, sc, CONFIGS["unbiased"], 3, spp=2)
    integ = load_dict({"type": "restirgi", **CONFIGS["unbiased"]})
    for fr in range(3):
        np.testing.assert_array_equal(integ.render_film(sc, seed=fr, spp=2), ref[fr], err_msg=f"frame {fr}")
    np.testing.assert_array_equal(integ.state("spatial"), orc.sres)


@pytest.mark.gpu
def test_restir_moving_camera_bit_exact(small_scene, oracle):
    """test-restir-dynamic.py: the sensor moves between frames; the temporal
    pass reprojects into the previous camera (prev_sensor, :247)."""
    from mtx import _abi, load_dict

    sc = small_scene.with_film(40, 24)
    cams = []
    for fr in range(3):
        c = _abi.Camera.from_buffer_copy(bytes(sc.camera))
        c.origin[0] += 0.03 * fr
        c.origin[2] -= 0.02 * fr
        cams.append(c)
    ref, orc = _oracle_frames(oracle, sc, CONFIGS["biased"], 3, cameras=cams)
    integ = load_dict({"type": "restirgi", **CONFIGS["biased"]})
    for fr in range(3):
        sc.camera = cams[fr]
        film = integ.render_film(sc, seed=fr, spp=1)
        np.testing.assert_array_equal(film, ref[fr], err_msg=f"frame {fr}")
    np.testing.assert_array_equal(integ.state("temporal"), orc.tres)


@pytest.mark.gpu
def test_restir_two_wavefront_split_bit_exact(small_scene, oracle):
    """A frame of >= 2^16 lanes runs stage A as two row halves on two
    wavefronts / streams (api.cpp render_restir): 384x216 (82,944 lanes), a
    moving camera, films and temporal reservoirs bit-exact vs the oracle."""
    from mtx import _abi, load_dict

    sc = small_scene.with_film(384, 216)
    assert sc.width * sc.height >= 1 << 16
    cams = []
    for fr in range(2):
        c = _abi.Camera.from_buffer_copy(bytes(sc.camera))
        c.origin[0] += 0.03 * fr
        cams.append(c)
    ref, orc = _oracle_frames(oracle, sc, CONFIGS["unbiased"], 2, cameras=cams)
    integ = load_dict({"type": "restirgi", **CONFIGS["unbiased"]})
    for fr in range(2):
        sc.camera = cams[fr]
        film = integ.render_film(sc, seed=fr, spp=1)
        np.testing.assert_array_equal(film, ref[fr], err_msg=f"frame {fr}")
    np.testing.assert_array_equal(integ.state("temporal"), orc.tres)


@pytest.mark.gpu
def test_restir_errors():
    from mtx import MtxError, load_dict, scene

    sc = scene.bedroom(32, 18, scale=0.02, tex_res=32)
    integ = load_dict({"type": "restirgi", "max_M_spatial": 500})
    with pytest.raises(MtxError):  # stage B without its stage A
        integ.render_film(sc, seed=0, spp=1, y0=4, stage="B")
    with pytest.raises(MtxError):
        integ.render_film(sc, seed=0, spp=1, stage="C")
    integ.render_film(sc, seed=0, spp=1)
    with pytest.raises(MtxError):
        integ.render_film(sc.with_film(16, 16), seed=1, spp=1)
    with pytest.raises(MtxError):
        integ.sample(sc, None, None)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["unbiased", "hemisphere_ss"])
def test_restir_row_bands_match_full_frame(small_scene, cfg):
    """a row-banded frame (stage A, halo exchange of samples and
    temporal reservoirs, stage B) reproduces the single-call frame: reservoir
    state bit-exact on every band's rows, stitched film up to the summation
    order of the band borders. Two contexts on one device stand in for two
    ranks; the exchange is the same row copy the RCCL path sends."""
    from mtx import distributed, load_dict
    from mtx._lib import Context

    sc = small_scene.with_film(40, 26)
    props = dict(CONFIGS[cfg])
    props["initial_search_radius"] = 6.0
    frames = 3
    full = load_dict({"type": "restirgi", **props})
    ref = [full.render_film(sc, seed=fr, spp=1) for fr in range(frames)]
    ref_state = {w: full.state(w) for w in ("temporal", "spatial", "radius")}

    bands = distributed.row_bands(sc.height, 2)
    ctxs = [Context(0), Context(0)]
    integs = [load_dict({"type": "restirgi", **props}) for _ in bands]
    halo = distributed.restir_halo(integs[0])
    io = [distributed.device_row_io(integs[k], sc, 1, ctxs[k]) for k in range(2)]
    for fr in range(frames):
        for k, (y0, y1) in enumerate(bands):
            integs[k].render_film(sc, seed=fr, spp=1, y0=y0, y1=y1, stage="A", ctx=ctxs[k])
        for k, (y0, y1) in enumerate(bands):
            _, _, recv_up, recv_down = distributed.halo_plan(y0, y1, sc.height, halo)
            other = 1 - k
            for which in ("sample", "temporal"):
                for row0, nrows in (recv_up, recv_down):
                    if nrows:
                        io[k][1](which, row0, io[other][0](which, row0, nrows))
        stitched = np.zeros_like(ref[fr])
        for k, (y0, y1) in enumerate(bands):
            stitched[y0:y1 + 2] += integs[k].render_film(sc, seed=fr, spp=1, y0=y0, y1=y1, stage="B", ctx=ctxs[k])
        np.testing.assert_allclose(stitched, ref[fr], rtol=2e-6, atol=1e-6, err_msg=f"frame {fr}")
    W = sc.width
    for k, (y0, y1) in enumerate(bands):
        for w in ("temporal", "spatial", "radius"):
            got = integs[k].state(w, ctx=ctxs[k])
            sl = slice(y0 * W, y1 * W)
            if w == "radius":
                assert np.array_equal(got[sl], ref_state[w][sl])
            else:
                assert np.array_equal(got[:, sl], ref_state[w][:, sl]), (k, w)
    for c in ctxs:
        c.close()
