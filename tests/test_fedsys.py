"""FedSys baseline: server-side selection rules and the summed-update model, single and multi rank."""
import numpy as np
import torch

from test_distributed_cpu import _free_port  # noqa: F401  (shared helper module)


def test_fedsys_select_rules(rt):
    fc = rt.FedSysConfig()
    fc.num_nodes, fc.perc_samples, fc.rand_sample = 20, 35, False
    fc.derive()
    assert fc.num_samples == 7 and fc.random_samples == 0          # int(20 * 0.35)
    sel = rt.fedsys_select(fc, list(range(1, 20)), 123)
    assert len(sel) == 7 and len(set(sel)) == 7 and sel == sorted(sel) and 0 not in sel
    fc.rand_sample = True
    fc.derive()
    assert fc.num_samples == 19 and fc.random_samples == 7           # wait for all, sample 7
    sel = rt.fedsys_select(fc, list(range(1, 20)), 123)
    assert len(sel) == 7 and all(1 <= s <= 19 for s in sel)         # with replacement


def test_fedsys_engine_sums_selected_updates():
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.fedsys import FedSysEngine

    cfg = RunConfig(num_nodes=8, dataset="creditcard", perc_samples=50, epsilon=0.0, device="cpu", seed=4)
    eng = FedSysEngine(cfg)
    seen = {}
    step = eng.task.step

    def spy(W, it, peers):  # record each worker's delta as the engine computes it
        d, q = step(W, it, peers)
        seen.update({p: d[i].clone() for i, p in enumerate(peers)})
        return d, q
    eng.task.step = spy
    errs = []
    for _ in range(6):
        W0 = eng.W.clone()
        r = eng.run_round()
        expect = W0 + torch.stack([seen[p] for p in r.selected]).double().sum(0)
        torch.testing.assert_close(eng.W, expect, rtol=0, atol=1e-12)
        assert len(r.selected) == 4 and 0 not in r.selected
        errs.append(r.test_error)
    assert errs[-1] <= errs[0] + 0.05
    assert len(eng.model_digest()) == 64


def test_fedsys_two_ranks_match_single():
    import os
    import sys

    import torch.multiprocessing as mp

    from test_distributed_cpu import ROOT

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    kw = dict(num_nodes=6, dataset="creditcard", perc_samples=50, device="cpu", seed=9, epsilon=5.0)
    ps = [ctx.Process(target=_fed_worker, args=(r, 2, port, kw, 4, q, ROOT)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.fedsys import FedSysEngine

    eng = FedSysEngine(RunConfig(**kw))
    for _ in range(4):
        eng.run_round()
    assert got[0] == got[1] == eng.model_digest()


def _fed_worker(rank, world, port, kw, rounds, q, root):
    import os
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, root)
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.fedsys import FedSysEngine

    comm = Comm.init(device="cpu")
    eng = FedSysEngine(RunConfig(**kw), comm)
    for _ in range(rounds):
        eng.run_round()
    q.put((rank, eng.model_digest()))
    comm.barrier()
    comm.shutdown()
