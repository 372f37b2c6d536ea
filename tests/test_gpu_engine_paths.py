"""Engine paths beyond the headline on the GPU: plain aggregation, RONI, churn, poisoners, FedSys,
creditcard/logreg -- each checked for chain validity and the exact-aggregation invariant."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    base = dict(num_nodes=12, dataset="mnist", seed=2, max_iterations=100, deterministic_time=True)
    base.update(kw)
    return BiscottiEngine(RunConfig(**base), Comm(device=torch.device("cuda", 0)))


def _run_exact(eng, rounds=4):
    seen = {}
    step = eng.task.step

    def spy(W, it, peers):  # record every peer's quantised update as the engine computes it
        d, q = step(W, it, peers)
        seen.update({(it, p): q[i].clone() for i, p in enumerate(peers)})
        return d, q
    eng.task.step = spy
    res = []
    for _ in range(rounds):
        W0 = eng.W.clone()
        r = eng.run_round()
        res.append(r)
        if not r.empty and eng.cfg.secure_agg:
            q = torch.stack([seen[(r.iteration, p)] for p in r.node_list])
            torch.testing.assert_close(eng.W, W0 + q.sum(0).double() / 10.0 ** eng.cfg.precision, rtol=0,
                                       atol=1e-12)
    ok, why = eng.fsm.chain.verify()
    assert ok, why
    eng.close()
    return res


def test_plain_aggregation_block_carries_updates():
    eng = _engine(secure_agg=False)
    res = _run_exact(eng)
    blk = eng.fsm.chain.latest()
    assert any(not r.empty for r in res)
    if len(blk.data.deltas):
        u = blk.data.deltas[0]
        assert len(u.delta) == 7850 and len(u.noised_delta) == 7850 and len(u.noise) == 7850


def test_roni_defense_on_gpu():
    res = _run_exact(_engine(defense="RONI"), 3)
    assert sum(not r.empty for r in res) >= 2


def test_churn_on_gpu():
    res = _run_exact(_engine(churn=0.2), 5)
    assert len(res) == 5


def test_poisoners_on_gpu():
    eng = _engine(num_nodes=20, poisoning=0.3)
    pois = {p for p in range(20) if eng.fsm.is_poisoner(p)}
    assert pois
    res = _run_exact(eng, 5)
    assert all(set(r.approved) <= set(range(20)) for r in res)


def test_creditcard_logreg_on_gpu():
    res = _run_exact(_engine(dataset="creditcard", num_nodes=8, num_verifiers=2, num_miners=2, num_noisers=1), 4)
    assert res[-1].test_error < 0.5


def test_fedsys_on_gpu():
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.fedsys import FedSysEngine

    eng = FedSysEngine(RunConfig(num_nodes=20, dataset="mnist", perc_samples=35, seed=1),
                       Comm(device=torch.device("cuda", 0)))
    errs = [eng.run_round().test_error for _ in range(6)]
    assert min(errs) < errs[0]
