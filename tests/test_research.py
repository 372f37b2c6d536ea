"""Research scripts of the reference (ML/code/*): linear model with top-k sparsified AdaGrad steps,
model inversion comparison, the bystander table (parity unpinned: synthetic / shipped credit data)."""
import numpy as np

from biscotti_amd import research as Rz


def test_linear_model_learns_and_sparsifies():
    m = Rz.LinearModel(*Rz.synthetic_regression(n=500, d=10, seed=1)[:2], seed=1)
    d = m.private_fun(0.3, np.zeros(10), batch_size=10)
    assert np.count_nonzero(d) == 3                      # only the top theta*d coordinates move
    out = Rz.run_linear(1.0, 400, 10, seed=2)
    assert out["curve"][-1][1] < 0.8 * out["curve"][0][1]   # AdaGrad at alpha 1e-2: slow but steady


def test_inversion_compare_and_bystanders_run():
    err = Rz.inversion_compare(Rz.train_victim(None, 200, seed=0))
    assert 0.0 <= err <= 1.0
    tab = Rz.bystander_table(iters=60, runs=1)
    assert set(tab) == {"no_dp", "eps1", "eps5"} and all(len(v["mean"]) == 4 for v in tab.values())
