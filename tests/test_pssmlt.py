"""PSSMLT restatement (pssmlt.py / pssmltsimple.py) — CPU checks of the oracle."""
import numpy as np


def test_pssmlt_chain_invariants(oracle, small_scene):
    from mtx import load_dict

    sc = small_scene.with_film(16, 9)
    integ = load_dict({"type": "pssmlt_simple", "iterations": 45})
    film, ch = oracle.pssmlt_render(sc, integ.render_args(sc, 1, 2), 45, chains=True)
    Lc, cw, off = ch[:, :3], ch[:, 3], ch[:, 4:6]
    assert np.isfinite(film).all()
    assert (cw > 0).all()
    assert ((off >= 0) & (off <= 1)).all()  # mutate_offset clamps to the pixel (pssmlt.py:250-254)
    assert (Lc >= 0).all()
    # aggregation iterations 41..44 put weight 4 x (0.25 x 4 pixels) per chain
    inner = film[..., 3].sum()
    assert abs(inner - 4 * 2 * 16 * 9) < 1e-3


def test_pssmlt_first_iteration_accepts(oracle, small_scene):
    """0/0 acceptance on the first iteration clamps to 1 (NaN-ignoring
    dr.clamp, pssmlt.py:137): every chain accepts, cw = 1."""
    from mtx import load_dict

    sc = small_scene.with_film(16, 9)
    integ = load_dict({"type": "pssmlt_simple", "iterations": 1})
    _, ch = oracle.pssmlt_render(sc, integ.render_args(sc, 3, 2), 1, chains=True)
    assert (ch[:, 3] == 1.0).all()
