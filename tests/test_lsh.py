"""LSH sieve (ML/code/logistic_aggregator.py:7-29): the exact neighbour query against a brute-force numpy
transcription of the reference's arithmetic, the LSH query as a subset of it, and the defence in the
round engine.  GPU kernels (LS1-LS3) against the CPU path: test_gpu_lsh below."""
import numpy as np
import pytest
import torch

from biscotti_amd.ops import lsh


def _sample(seed=0, d=5):
    rng = np.random.default_rng(seed)
    good = (rng.random((50, d)) - 0.5) * 2          # the reference's own demo data (__main__)
    attackers = np.repeat(rng.random((1, d)) + 0.5, 10, axis=0) + 1e-4 * rng.random((10, d))
    return np.vstack((good, attackers))


def _brute(deltas, thr):
    c = deltas - deltas.mean(0)
    d2 = ((c[:, None, :] - c[None, :, :]) ** 2).sum(-1)
    cnt = (d2 < thr).sum(1)
    return (deltas / cnt[:, None]).sum(0), cnt


def test_exact_sieve_matches_reference_arithmetic():
    X = _sample()
    ref_grad, ref_cnt = _brute(X, 1.0 / X.shape[1])
    grad, cnt = lsh.lsh_sieve(torch.from_numpy(X).float(), tables=0)
    assert cnt.tolist() == ref_cnt.tolist()
    assert (ref_cnt[-10:] == 10).all()                # the sybil cluster shares one update's weight
    np.testing.assert_allclose(grad.numpy(), ref_grad, rtol=1e-5, atol=1e-5)


def test_lsh_query_finds_a_subset_of_true_neighbours():
    X = torch.from_numpy(_sample(1, d=64)).float()
    exact = lsh.neighbour_counts(X, 1.0 / 64, [list(range(60))], tables=0)[0]
    approx = lsh.neighbour_counts(X, 1.0 / 64, [list(range(60))], tables=4, bits=8)[0]
    assert (approx >= 1).all() and (approx <= exact).all()
    assert (approx[-10:] == 10).all()                 # near-identical rows always collide


def test_lsh_defense_rounds_keep_a_valid_chain():
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    eng = BiscottiEngine(RunConfig(num_nodes=8, dataset="creditcard", num_verifiers=2, num_miners=2, num_noisers=1,
                                   device="cpu", seed=3, defense="LSH", deterministic_time=True))
    res = [eng.run_round() for _ in range(3)]
    assert sum(not r.empty for r in res) >= 2
    assert all(set(r.node_list) <= set(r.approved) for r in res)
    assert eng.fsm.chain.verify()[0]
    eng.close()


@pytest.mark.gpu
def test_gpu_lsh_kernels_match_cpu():
    X = torch.from_numpy(_sample(2, d=300)).float()
    for tables in (0, 4):
        g_cpu, c_cpu = lsh.lsh_sieve(X, tables=tables, bits=10, seed=5)
        g_gpu, c_gpu = lsh.lsh_sieve(X.cuda(), tables=tables, bits=10, seed=5)
        assert c_gpu.tolist() == c_cpu.tolist(), tables
        torch.testing.assert_close(g_gpu.cpu(), g_cpu, rtol=1e-9, atol=1e-9)
    P = lsh.planes(4, 10, 300, 5, "cpu")
    mu = X.mean(0)
    assert torch.equal(lsh.codes(X.cuda(), mu.cuda(), P.cuda(), 4, 10).cpu(), lsh.codes(X, mu, P, 4, 10))
