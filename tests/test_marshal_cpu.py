"""Host logic of BundleAdjuster.set_problem_from's marshalling cache: the marshalled
arguments are cached on the problem object only when every field was used as it is, so in-place
edits of a field that had to be converted (wrong dtype, non-contiguous) are never lost."""
import numpy as np


def _setup(monkeypatch):
    from rsvio.ba import BundleAdjuster
    calls = []
    ba = object.__new__(BundleAdjuster)
    monkeypatch.setattr(BundleAdjuster, "_set", lambda self, keep, args: calls.append((keep, args)))
    return ba, calls


def _problem(obs_lm_dtype=np.int32, p_w_f32=False):
    from rsvio import synthetic as S
    p = S.ba_problem(n_kf=4, n_lm=30, kf_per_lm=3, seed=1, init_seed=2)
    object.__setattr__(p, "obs_lm", p.obs_lm.astype(obs_lm_dtype))
    if p_w_f32:
        object.__setattr__(p, "p_W", p.p_W.astype(np.float32))
    return p


def test_cached_when_fields_are_used_as_they_are(monkeypatch):
    ba, calls = _setup(monkeypatch)
    p = _problem()
    ba.set_problem_from(p)
    ba.set_problem_from(p)
    assert calls[0][1] == calls[1][1]          # the same pointers: the cache was used
    assert "_rsvio_marshal" in p.__dict__
    p.p_W[0, 0] += 1.0                          # in-place edit: seen through the cached view
    assert calls[1][0][2][0, 0] == p.p_W[0, 0]


def test_converted_field_is_remarshalled_every_call(monkeypatch):
    for kw in ({"obs_lm_dtype": np.int64}, {"p_w_f32": True}):
        ba, calls = _setup(monkeypatch)
        p = _problem(**kw)
        ba.set_problem_from(p)
        assert "_rsvio_marshal" not in p.__dict__
        if "p_w_f32" in kw:
            p.p_W[0, 0] += 1.0
            ba.set_problem_from(p)
            assert calls[1][0][2][0, 0] == np.float64(p.p_W[0, 0])   # the edit reached the upload
        else:
            p.obs_lm[0] = 7
            ba.set_problem_from(p)
            assert calls[1][0][3][0] == 7
