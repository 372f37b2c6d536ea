"""gfx950 learning-side kernels vs the CPU reference path (same Philox streams, fp32/fp64 refs)."""
import numpy as np
import pytest
import torch

from biscotti_amd.ops import ml as K

pytestmark = pytest.mark.gpu


def _fed(P=6, n=40, d_in=784, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn((P * n, d_in), generator=g)
    y = torch.randint(0, 10, (P * n,), generator=g, dtype=torch.int32)
    off = torch.arange(P, dtype=torch.int64) * n
    nt = torch.full((P,), n, dtype=torch.int32)
    pid = torch.arange(P, dtype=torch.int32) * 7 + 3
    W = torch.randn(10 * d_in + 10, generator=g, dtype=torch.float64) * 0.05
    return X, y, off, nt, pid, W


def test_softmax_step_matches_reference():
    X, y, off, nt, pid, W = _fed()
    d_ref, q_ref, l_ref = K.softmax_step(X, y, off, nt, pid, W, 784, 10, 10, 1234, 5)
    c = lambda t: t.cuda()
    d_gpu, q_gpu, l_gpu = K.softmax_step(c(X), c(y), c(off), c(nt), c(pid), c(W), 784, 10, 10, 1234, 5)
    torch.testing.assert_close(d_gpu.cpu(), d_ref, rtol=2e-4, atol=2e-6)
    torch.testing.assert_close(l_gpu.cpu(), l_ref, rtol=1e-4, atol=1e-5)
    assert (q_gpu.cpu() - q_ref).abs().max() <= 1


def test_softmax_step_resident_indexing_matches_row_indexing():
    """lo >= 0: off / ntrain indexed by pid - lo over all local peers (a subset, out of order)."""
    X, y, off, nt, _, W = _fed()
    lo = 40
    pid_all = torch.arange(lo, lo + off.numel(), dtype=torch.int32)
    sel = torch.tensor([3, 0, 5, 2], dtype=torch.long)
    c = lambda t: t.cuda()
    d_row, q_row, l_row = K.softmax_step(c(X), c(y), c(off[sel]), c(nt[sel]), c(pid_all[sel]), c(W), 784, 10, 10, 99, 2)
    d_res, q_res, l_res = K.softmax_step(c(X), c(y), c(off), c(nt), c(pid_all[sel]), c(W), 784, 10, 10, 99, 2, lo=lo)
    assert torch.equal(d_row, d_res) and torch.equal(q_row, q_res) and torch.equal(l_row, l_res)
    d_cpu, _, _ = K.softmax_step(X, y, off, nt, pid_all[sel], W, 784, 10, 10, 99, 2, lo=lo)
    torch.testing.assert_close(d_res.cpu(), d_cpu, rtol=2e-4, atol=2e-6)


@pytest.mark.parametrize("d_in,d_out", [(8742, 2), (2500, 12)])
def test_softmax_step_k_tiled_matches_reference(d_in, d_out):
    """K-tiled local step (features staged through LDS in 1024-wide tiles): LFW-sized 62x47x3 inputs."""
    g = torch.Generator().manual_seed(d_in)
    P, n = 6, 40
    X = torch.rand((P * n, d_in), generator=g)
    y = torch.randint(0, d_out, (P * n,), generator=g, dtype=torch.int32)
    off = torch.arange(P, dtype=torch.int64) * n
    nt = torch.full((P,), n, dtype=torch.int32)
    pid = torch.arange(P, dtype=torch.int32) * 5 + 1
    W = torch.randn(d_out * d_in + d_out, generator=g, dtype=torch.float64) * 0.01
    d_ref, q_ref, l_ref = K.softmax_step(X, y, off, nt, pid, W, d_in, d_out, 10, 77, 3)
    c = lambda t: t.cuda()
    d_gpu, q_gpu, l_gpu = K.softmax_step(c(X), c(y), c(off), c(nt), c(pid), c(W), d_in, d_out, 10, 77, 3)
    torch.testing.assert_close(d_gpu.cpu(), d_ref, rtol=5e-4, atol=5e-6)
    torch.testing.assert_close(l_gpu.cpu(), l_ref, rtol=1e-4, atol=1e-5)
    assert (q_gpu.cpu() - q_ref).abs().max() <= 1


def test_lfw_ledger_rounds_on_gpu():
    """The long-parameter-vector ledger (LFW maleness softmax, d = 17486, 1749 chunks): exact secure
    aggregation and a valid chain."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    cfg = RunConfig(num_nodes=20, dataset="lfw", seed=4, max_iterations=100, deterministic_time=True)
    eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
    assert eng.d == 17486
    res = []
    for _ in range(3):
        W0 = eng.W.clone()
        r = eng.run_round()
        res.append(r)
        if not r.empty:
            _, q = eng.task.step(W0, r.iteration, sorted(r.node_list))
            torch.testing.assert_close(eng.W, W0 + q.sum(0).double() / 1e4, rtol=0, atol=1e-12)
    ok, why = eng.fsm.chain.verify()
    eng.close()
    assert ok, why
    assert sum(not r.empty for r in res) >= 2


def test_softmax_step_clips_large_gradients():
    X, y, off, nt, pid, W = _fed(P=3)
    X = X * 1e3  # huge activations -> gradient norm far above 100
    d_gpu, _, _ = K.softmax_step(X.cuda(), y.cuda(), off.cuda(), nt.cuda(), pid.cuda(), W.cuda(), 784, 10, 10, 9, 0)
    norms = d_gpu.double().norm(dim=1)
    assert torch.all(norms <= 100.0 + 1e-3) and torch.all(norms > 99.0)


def test_logreg_step_matches_reference():
    g = torch.Generator().manual_seed(1)
    X = torch.randn((300, 25), generator=g, dtype=torch.float64)
    y = torch.where(torch.rand(300, generator=g) > 0.5, 1.0, -1.0).double()
    off = torch.tensor([0, 100, 200], dtype=torch.int64)
    nr = torch.tensor([100, 100, 100], dtype=torch.int32)
    pid = torch.tensor([0, 1, 2], dtype=torch.int32)
    W = torch.randn(25, generator=g, dtype=torch.float64) * 0.1
    calls = torch.tensor([1, 2, 3], dtype=torch.int32)
    sigma = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
    ref = K.logreg_step(X, y, off, nr, pid, W, 10, 77, calls, 1e-2, 1e-2, sigma)
    c = lambda t: t.cuda()
    got = K.logreg_step(c(X), c(y), c(off), c(nr), c(pid), c(W), 10, 77, c(calls), 1e-2, 1e-2, c(sigma))
    torch.testing.assert_close(got[0].cpu(), ref[0], rtol=1e-4, atol=1e-6)


def test_dp_noise_matches_reference():
    delta = torch.randn((5, 7850))
    noisers = torch.tensor([[1, 2], [2, 3], [1, 4], [0, 9], [5, 6]], dtype=torch.int32)
    scales = torch.full((5, 2), -0.77)
    scales[3, 1] = 0.0  # colluding noiser
    ref = K.dp_noise(delta, noisers, scales, 42, 13)
    got = K.dp_noise(delta.cuda(), noisers.cuda(), scales.cuda(), 42, 13).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    # same noiser + iteration -> same noise vector for every worker (pre-sampled samples semantics)
    n01 = got[0] - delta[0]
    n21 = got[2] - delta[2]
    assert not torch.allclose(n01, n21)


def test_krum_matches_reference():
    g = torch.Generator().manual_seed(3)
    X = torch.randn((70, 7850), generator=g) * 0.1
    X[60:] += 3.0  # outliers
    acc_ref, sc_ref = K.krum(X, 35, 35)
    acc, sc = K.krum(X.cuda(), 35, 35)
    torch.testing.assert_close(sc.cpu(), sc_ref, rtol=1e-9, atol=1e-6)
    assert torch.equal(acc.cpu(), acc_ref)
    assert not acc.cpu()[60:].any()


def test_eval_error_matches_reference():
    X, y, off, nt, pid, W = _fed(P=1, n=2000)
    ref = K.eval_error(X, y, W, 784, 10)
    got = K.eval_error(X.cuda(), y.cuda(), W.cuda(), 784, 10)
    assert abs(ref - got) <= 1.0 / 2000


def test_recover_exact(rt):
    rng = np.random.default_rng(0)
    nch, poly = 50, 10
    coeffs = rng.integers(-10**7, 10**7, size=(nch, poly))
    xs = np.arange(-10, 11)
    ys = np.stack([[sum(int(c) * int(x) ** j for j, c in enumerate(row)) for x in xs] for row in coeffs])
    W = torch.zeros(nch * poly - 3, dtype=torch.float64)
    Wn, got, st = K.recover(torch.from_numpy(ys).cuda(), torch.from_numpy(xs.astype(np.int32)).cuda(), poly,
                            W.numel(), W.cuda(), 1e4)
    assert st.cpu().all()
    np.testing.assert_array_equal(got.cpu().numpy(), coeffs)
    np.testing.assert_allclose(Wn.cpu().numpy(), coeffs.reshape(-1)[: W.numel()] / 1e4)
    bad = ys.copy()
    bad[3, 5] += 1
    _, _, st2 = K.recover(torch.from_numpy(bad).cuda(), torch.from_numpy(xs.astype(np.int32)).cuda(), poly,
                          W.numel(), W.cuda(), 1e4)
    assert st2.cpu()[3] == 0 and st2.cpu().sum() == nch - 1
    # two miners only (x in -10..-4 and 4..10): still exact
    sel = list(range(0, 7)) + list(range(14, 21))
    _, got3, st3 = K.recover(torch.from_numpy(ys[:, sel].copy()).cuda(),
                             torch.from_numpy(xs[sel].astype(np.int32)).cuda(), poly, W.numel(), W.cuda(), 1e4)
    assert st3.cpu().all()
    np.testing.assert_array_equal(got3.cpu().numpy(), coeffs)


@pytest.mark.parametrize("cols", [list(range(21)), list(range(0, 7)) + list(range(14, 21))])
def test_recover_rows_fused_weights(cols):
    """k_recover_w (share sums fused, precomputed exact weights) against the 128-bit Newton kernel's
    contract: exact coefficients for consistent shares, status 0 for a tampered share, masked rows
    left out of the sums."""
    rng = np.random.default_rng(1)
    R, nch, poly, T = 6, 785, 10, 21
    per = rng.integers(-3 * 10**6, 3 * 10**6, size=(R, nch, poly))
    xs_all = np.arange(-10, 11)
    pw = xs_all[None, :] ** np.arange(poly)[:, None]             # [poly, 21]
    ys = np.einsum("rkj,jx->rkx", per, pw).astype(np.int64)       # shares of every row
    mask = np.array([1, 0, 1, 1, 0, 1], np.int32)
    tot = per[mask.astype(bool)].sum(0)                           # [nch, poly]
    xs = xs_all[cols]
    w = K.recovery_weights(xs.tolist(), poly)
    A = torch.from_numpy(w["A"].reshape(-1)).cuda()
    basis = torch.tensor(w["basis"], dtype=torch.int32).cuda()
    ys_t = torch.from_numpy(ys).cuda()
    W = torch.zeros(7850, dtype=torch.float64).cuda()
    ycols = torch.tensor(cols, dtype=torch.int32).cuda()
    xs_t = torch.from_numpy(xs.astype(np.int32)).cuda()
    Wn, got, st, agg = K.recover_rows(ys_t, torch.from_numpy(mask).cuda(), ycols, xs_t, w, A, basis, poly, 7850, W)
    assert st.cpu().all()
    np.testing.assert_array_equal(got.cpu().numpy(), tot)
    np.testing.assert_array_equal(agg.cpu().numpy(), ys[mask.astype(bool)].sum(0)[:, cols])
    np.testing.assert_allclose(Wn.cpu().numpy(), tot.reshape(-1)[:7850] / 1e4)
    bad = ys.copy()
    bad[2, 7, cols[3]] += 1
    _, _, st2, _ = K.recover_rows(torch.from_numpy(bad).cuda(), torch.from_numpy(mask).cuda(), ycols, xs_t, w, A,
                                  basis, poly, 7850, W)
    assert st2.cpu()[7] == 0 and st2.cpu().sum() == nch - 1


@pytest.mark.parametrize("ablation", ["", "no_pipeline"])
def test_engine_rounds_on_gpu(ablation):
    """Whole GPU round pipeline (speculative shares on the CU-masked stream, async commitments,
    pipelined round heads): each block's model is EXACTLY the old model plus the sum of the
    included workers' quantised updates, recomputed independently through the Philox step."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    cfg = RunConfig(num_nodes=12, dataset="mnist", seed=3, max_iterations=100, ablation=ablation)
    pre_step = not ablation
    eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
    res = []
    for _ in range(5):
        W0 = eng.W.clone()
        r = eng.run_round()
        res.append(r)
        if r.empty:
            torch.testing.assert_close(eng.W, W0, rtol=0, atol=0)
            continue
        _, q = eng.task.step(W0, r.iteration, sorted(r.node_list))
        expect = W0 + q.sum(0).double() / 10.0 ** cfg.precision
        torch.testing.assert_close(eng.W, expect, rtol=0, atol=1e-12)
    ok, why = eng.fsm.chain.verify()
    assert ok, why
    assert sum(not r.empty for r in res) >= 3
    assert min(r.test_error for r in res) < 0.8
    # the device-side aggregation queued behind Krum was adopted (and matched the exact sums above)
    assert eng.stats.get("device_aggregations", 0) >= 3
    assert eng.stats["audit_failures"] == 0
    # the next round's local step queued behind the recovery was adopted (and the blocks above match
    # the independently recomputed step)
    assert (eng.stats.get("pre_steps", 0) >= 1) if pre_step else "pre_steps" not in eng.stats
    eng.close()


def test_pre_gram_and_early_vrf_keep_the_chain():
    """The Krum Gram queued with the pre-step (rows = every local peer, on its own stream), the VRF
    outputs started at block build and the next round's share MSM launched from fsm.successor(block)
    before the audit give byte-identical chains to the in-round Gram (rows = workers), the VRF
    submitted by the head and the MSM launched by the head -- with poisoners, so Krum's selection
    decides the blocks."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    chains, stats = [], []
    for on in (True, False):
        cfg = RunConfig(num_nodes=20, dataset="mnist", seed=4, max_iterations=100, deterministic_time=True,
                        poisoning=0.3, epsilon=1.0, ablation="" if on else "no_pipeline")
        eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
        for _ in range(6):
            eng.run_round()
        chains.append([bytes(eng.fsm.chain.block(i).hash) for i in range(len(eng.fsm.chain))])
        stats.append(dict(eng.stats))
        eng.close()
    assert chains[0] == chains[1]
    assert stats[0].get("early_vrf", 0) >= 4 and "early_vrf" not in stats[1]
    assert stats[0].get("spec_head", 0) >= 4 and "spec_head" not in stats[1]
    assert stats[0].get("device_aggregations", 0) >= 4


@pytest.mark.parametrize("extra", ["", "spec_tight"])
def test_early_front_keeps_the_chain(extra):
    """The next round's front (noiser lottery, Krum launch, the aggregation queued behind the selection) started
    right after the previous round's block build (the speculative front), or at the previous round's commit
    (no_spec_front), gives the chain of running it at the round's own start (no_early_front), with poisoners
    (Krum's selection decides the blocks) and with spec_tight (speculative misses: the host path aggregates behind
    an early-launched selection)."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    chains, stats = [], []
    for abl in (extra, ",".join(a for a in (extra, "no_early_front") if a),
                ",".join(a for a in (extra, "no_spec_front") if a)):
        cfg = RunConfig(num_nodes=30, dataset="mnist", seed=5, max_iterations=100, deterministic_time=True,
                        poisoning=0.3, epsilon=1.0, ablation=abl)
        eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
        for k in range(10):
            eng.run_round(front=k != 4, last=k == 9)   # one round without a front: the next starts its own
        eng.drain()
        ok, why = eng.fsm.chain.verify()
        assert ok, why
        chains.append([bytes(eng.fsm.chain.block(i).hash) for i in range(len(eng.fsm.chain))])
        stats.append(dict(eng.stats))
        eng.close()
    assert chains[0] == chains[1] == chains[2]
    assert stats[0].get("early_fronts", 0) == 8 and "early_fronts" not in stats[1]
    assert stats[2].get("early_fronts", 0) == 8 and "spec_fronts" not in stats[2]
    assert stats[0].get("spec_fronts", 0) >= 6 and "spec_front_drops" not in stats[0], stats[0]
    assert stats[0]["audit_failures"] == 0
    if extra:   # a miss aggregates on the host-decided path
        assert stats[0].get("spec_misses", 0) > 0, stats[0]
        assert stats[0].get("device_aggregations", 0) + stats[0]["spec_misses"] >= 8, stats[0]
    else:
        assert stats[0].get("device_aggregations", 0) >= 6, stats[0]


def test_spec_front_dropped_when_the_block_changes(monkeypatch):
    """A speculative front whose block is not the one committed -- round 3's block replaced by an empty one after
    its build, as a failed aggregate audit does -- is dropped (its generator stopped, its VRF job joined later) and
    the round opened afresh from the already begun plan: the chain is the one of fronts launched at the commit
    (no_spec_front)."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine
    from biscotti_amd.protocol.secagg import SecAggMixin

    real = SecAggMixin._finish_secagg

    def empty_at_3(self, plan, *a):
        blk = real(self, plan, *a)
        return None if plan.iteration == 3 else blk
    monkeypatch.setattr(SecAggMixin, "_finish_secagg", empty_at_3)
    chains, stats = [], []
    for abl in ("", "no_spec_front"):
        cfg = RunConfig(num_nodes=30, dataset="mnist", seed=5, max_iterations=100, deterministic_time=True,
                        poisoning=0.3, epsilon=1.0, ablation=abl)
        eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
        for k in range(8):
            eng.run_round(last=k == 7)
        eng.drain()
        ok, why = eng.fsm.chain.verify()
        assert ok, why
        chains.append([bytes(eng.fsm.chain.block(i).hash) for i in range(len(eng.fsm.chain))])
        stats.append(dict(eng.stats))
        eng.close()
    assert chains[0] == chains[1]
    assert stats[0].get("spec_front_drops", 0) == 1 and stats[0].get("spec_fronts", 0) >= 4, stats[0]
    assert "spec_fronts" not in stats[1]


def test_last_round_vrf_proofs_on_the_host():
    """The run's last round (remaining = 1) proves its VRF proofs on the host threads (vrf_proofs_async,
    AVX-512 IFMA batches) while the rounds before it go to the device prover: every proof is made, the drain
    joins both, and the chain is the one of a run without the hint."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    chains, stats = [], []
    for hint in (True, False):
        cfg = RunConfig(num_nodes=20, dataset="mnist", seed=6, max_iterations=100, deterministic_time=True)
        eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
        for k in range(6):
            eng.run_round(last=k == 5, remaining=6 - k if hint else None)
        eng.drain()
        chains.append([bytes(eng.fsm.chain.block(i).hash) for i in range(len(eng.fsm.chain))])
        stats.append(dict(eng.stats))
        eng.close()
    assert chains[0] == chains[1]
    assert stats[0].get("vrf_host_proofs", 0) > 0 and "vrf_host_proofs" not in stats[1]
    # the same proofs in total: the device's count plus the host's equals the all-device run's
    assert stats[0]["vrf_device_proofs"] + stats[0]["vrf_host_proofs"] == stats[1]["vrf_device_proofs"]


@pytest.mark.parametrize("U,n,V", [(94, 70, 3), (150, 140, 5), (256, 256, 3), (300, 200, 26)])
def test_krum_committee_matches_reference(U, n, V):
    """Committee Multi-Krum (one Gram over the candidate rows, per-verifier inboxes, vote and leader
    cap) against the fp64 torch reference, incl. inboxes of 140 and 256 updates (200-peer runs)."""
    g = torch.Generator().manual_seed(U + n + V)
    X = torch.randn((U, 7850), generator=g) * 0.1
    bad = torch.randperm(U, generator=g)[: U // 5]
    X[bad] += 0.5 * torch.randn((1, 7850), generator=g)        # a tight cluster of outliers
    inbox = torch.stack([torch.sort(torch.randperm(U, generator=g)[:n]).values for _ in range(V)]).int()
    rank = torch.randperm(U, generator=g).int()
    rank[torch.randperm(U, generator=g)[:3]] = -1                # rows that did not submit
    clip = n // 2
    need, cap = V // 2, max(2, n // 4)
    acc_ref, node_ref = K.krum_committee_async(X, inbox, n - clip, n - clip, need, rank, cap)()
    acc, node = K.krum_committee_async(X.cuda(), inbox.cuda(), n - clip, n - clip, need, rank.cuda(), cap)()
    assert torch.equal(acc, acc_ref)
    assert torch.equal(node, node_ref)
    assert int(node.sum()) <= cap
    # the outliers are rejected by every verifier that saw them
    for v in range(V):
        rows = inbox[v].long()
        assert not acc[v][torch.isin(rows, bad)].any()


@pytest.mark.parametrize("U1,N,nn", [(94, 100, 2), (60, 64, 3)])
def test_krum_committee_noise_aware_matches_explicit(U1, N, nn):
    """Phase-1 Gram over [deltas; noise vectors] + phase-2 assembly gives the same committee decisions as
    Krum over the explicitly noised rows (fp64 reference), incl. a colluding noiser (scale 0)."""
    g = torch.Generator().manual_seed(U1 + N)
    D = 7850
    delta = (torch.randn((U1, D), generator=g) * 0.05).float()
    bad = torch.arange(U1 - U1 // 4, U1)
    delta[bad] += 0.3 * torch.randn((1, D), generator=g)
    tbl = torch.randn((N, 100, D), generator=g).float()
    it = 37
    nz = torch.randint(0, N, (U1, nn), generator=g).int()
    sc = torch.full((U1, nn), -0.76, dtype=torch.float32)
    sc[5, 0] = 0.0
    X64 = delta.double() + (sc.double()[:, :, None] * tbl[:, it].double()[nz.long()]).sum(1) / nn
    n, V = min(70, U1 - 4), 3
    inbox = torch.stack([torch.sort(torch.randperm(U1, generator=g)[:n]).values for _ in range(V)]).int()
    rank = torch.randperm(U1, generator=g).int()
    clip = n // 2
    acc_ref, node_ref = K.krum_committee_async(X64, inbox, n - clip, n - clip, 1, rank, 20)()
    pre = K.gram_stacked_async(delta.cuda(), tbl.cuda()[:, it, :])
    acc, node = K.krum_committee_noise_async(pre, nz.cuda(), sc.cuda(), inbox.cuda(), n - clip, n - clip, 1,
                                             rank.cuda(), 20)()
    assert torch.equal(acc, acc_ref)
    assert torch.equal(node, node_ref)
    if K.noise_tables_by_value(U1 * nn, n):
        # the host tables in the rows kernel's argument block (the one-rank round's path): the same decisions
        acc2, node2 = K.krum_committee_noise_async(pre, nz.numpy(), sc.numpy(), inbox.cuda(), n - clip, n - clip, 1,
                                                   rank.cuda(), 20)()
        assert torch.equal(acc2, acc_ref)
        assert torch.equal(node2, node_ref)


def test_krum_committee_single_verifier_equals_krum():
    g = torch.Generator().manual_seed(5)
    X = torch.randn((70, 7850), generator=g) * 0.1
    X[60:] += 3.0
    acc_ref, _ = K.krum(X, 35, 35)
    inbox = torch.arange(70, dtype=torch.int32)[None]
    acc, node = K.krum_committee_async(X.cuda(), inbox.cuda(), 35, 35, 1, torch.arange(70, dtype=torch.int32).cuda(),
                                       0)()
    assert torch.equal(acc[0], acc_ref)
    assert torch.equal(node, acc_ref)


def test_eval_errors_two_sets_one_launch():
    """Test error and attack rate from one MFMA kernel launch, against the fp32 torch reference."""
    X, y, off, nt, pid, W = _fed(P=1, n=2347)
    split = 2000
    ref_a = K.eval_error(X[:split], y[:split], W, 784, 10)
    ref_b = K.eval_error(X[split:], y[split:], W, 784, 10)
    a, b = K.eval_errors_async(X.cuda(), y.cuda(), split, W.cuda(), 784, 10)()
    assert abs(a - ref_a) <= 1.0 / split and abs(b - ref_b) <= 1.0 / (2347 - split)
    # rows not a multiple of the 16-row tile, no transform
    Xs, ys_ = X[:37], y[:37]
    assert abs(K.eval_error(Xs.cuda(), ys_.cuda(), W.cuda(), 784, 10, transform=False)
               - K.eval_error(Xs, ys_, W, 784, 10, transform=False)) <= 1.0 / 37


def test_noise_table_matches_on_the_fly():
    """The resident noise table gives bit-identical noised deltas to per-round generation."""
    delta = torch.randn((7, 7850)).cuda()
    noisers = torch.tensor([[1, 2], [2, 3], [1, 4], [0, 9], [5, 6], [11, 3], [0, 0]], dtype=torch.int32).cuda()
    scales = torch.full((7, 2), -0.77).cuda()
    scales[3, 1] = 0.0
    tbl = K.noise_table(12, 7850, 42, "cuda")
    for it in (0, 13, 113):
        a = K.dp_noise(delta, noisers, scales, 42, it)
        b = K.dp_noise(delta, noisers, scales, 42, it, table=tbl)
        assert torch.equal(a, b), it
    ref = K.noise_vector(5, 13, 7850, 42)
    np.testing.assert_allclose(tbl[5, 13].cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


def test_noise_table_fused_row_gather():
    """rows= gathers the verifiers' inbox straight out of the noise kernel."""
    delta = torch.randn((6, 300)).cuda()
    noisers = torch.tensor([[1, 2], [2, 3], [1, 4], [0, 5], [5, 3], [4, 0]], dtype=torch.int32).cuda()
    scales = torch.full((6, 2), 0.5).cuda()
    tbl = K.noise_table(6, 300, 7, "cuda")
    full = K.dp_noise(delta, noisers, scales, 7, 4, table=tbl)
    rows = torch.tensor([4, 0, 5, 2], dtype=torch.int32).cuda()
    got = K.dp_noise(delta, noisers, scales, 7, 4, table=tbl, rows=rows)
    assert torch.equal(got, full[rows.long()])


@pytest.mark.parametrize("U,n,V", [(500, 400, 3), (1300, 700, 4)])
def test_krum_committee_large_inboxes(U, n, V):
    """Committees past the LDS fast path (inbox > 256 updates, > 1024 candidate rows; the reference's Krum
    has no size limit, client_obj.py:114-143): rows sorted in LDS + workspace vote, against the fp64
    reference (BLAS Gram here: the test's rows have no near-ties)."""
    g = torch.Generator().manual_seed(U + n)
    X = torch.randn((U, 7850), generator=g) * 0.1
    bad = torch.randperm(U, generator=g)[: U // 5]
    X[bad] += 0.5 * torch.randn((1, 7850), generator=g)
    inbox = torch.stack([torch.sort(torch.randperm(U, generator=g)[:n]).values for _ in range(V)]).int()
    rank = torch.randperm(U, generator=g).int()
    rank[torch.randperm(U, generator=g)[:5]] = -1
    clip = n // 2
    need, cap = V // 2, n // 3
    Xd = X.double()
    acc_ref, node_ref = K._committee_host(None, inbox, n - clip, n - clip, need, rank, cap, G=Xd @ Xd.T)
    acc, node = K.krum_committee_async(X.cuda(), inbox.cuda(), n - clip, n - clip, need, rank.cuda(), cap)()
    assert torch.equal(acc, acc_ref)
    assert torch.equal(node, node_ref)
    for v in range(V):
        assert not acc[v][torch.isin(inbox[v].long(), bad)].any()


def test_krum_committee_noise_aware_large_inbox():
    """Noise-aware assembly with an inbox of 400 (sorted-row path) against explicitly noised rows."""
    g = torch.Generator().manual_seed(77)
    U1, N, nn, D, it = 600, 300, 2, 7850, 1
    delta = (torch.randn((U1, D), generator=g) * 0.05).float()
    delta[-100:] += 0.3 * torch.randn((1, D), generator=g)
    tbl = torch.randn((N, 2, D), generator=g).float()
    nz = torch.randint(0, N, (U1, nn), generator=g).int()
    sc = torch.full((U1, nn), -0.76, dtype=torch.float32)
    X64 = delta.double() + (sc.double()[:, :, None] * tbl[:, it].double()[nz.long()]).sum(1) / nn
    n, V = 400, 3
    inbox = torch.stack([torch.sort(torch.randperm(U1, generator=g)[:n]).values for _ in range(V)]).int()
    rank = torch.randperm(U1, generator=g).int()
    clip = n // 2
    acc_ref, node_ref = K._committee_host(None, inbox, n - clip, n - clip, 1, rank, 60, G=X64 @ X64.T)
    pre = K.gram_stacked_async(delta.cuda(), tbl.cuda()[:, it, :])
    acc, node = K.krum_committee_noise_async(pre, nz.cuda(), sc.cuda(), inbox.cuda(), n - clip, n - clip, 1,
                                             rank.cuda(), 60)()
    assert torch.equal(acc, acc_ref)
    assert torch.equal(node, node_ref)


def test_eval_errors_cached_tiles_match_reference():
    """k_eval_error_t on the cached pre-transformed tiles (the engine's evaluation): the same error counts
    as the fp32 torch reference, for a row count that is not a multiple of the 16-row tile."""
    X, y, off, nt, pid, W = _fed(P=1, n=2347)
    split = 2000
    ref_a = K.eval_error(X[:split], y[:split], W, 784, 10)
    ref_b = K.eval_error(X[split:], y[split:], W, 784, 10)
    Xc = X.cuda()
    Xt = K.eval_tiles(Xc, transform=True)
    assert tuple(Xt.shape) == ((2347 + 15) // 16, 196, 64)
    a, b = K.eval_errors_async(Xc, y.cuda(), split, W.cuda(), 784, 10, Xt=Xt)()
    assert abs(a - ref_a) <= 1.0 / split and abs(b - ref_b) <= 1.0 / (2347 - split)
    a0, b0 = K.eval_errors_async(Xc, y.cuda(), split, W.cuda(), 784, 10)()   # the gather kernel
    assert abs(a - a0) <= 1.0 / split and abs(b - b0) <= 1.0 / (2347 - split)


def test_eval_errors_cached_tiles_repeated_launches():
    """The cached-tile evaluation resets its own counters (its last tile writes the host copy and re-zeroes
    them): back-to-back launches over the rotating buffers, each with a different model, each match the
    reference, including results read only after later launches were queued."""
    X, y, off, nt, pid, W = _fed(P=1, n=1000)
    split = 700
    Xc, yc = X.cuda(), y.cuda()
    Xt = K.eval_tiles(Xc, transform=True)
    g = torch.Generator().manual_seed(5)
    Ws = [W + 0.05 * k * torch.randn(W.shape, generator=g, dtype=W.dtype) for k in range(7)]
    pending = [K.eval_errors_async(Xc, yc, split, Wk.cuda(), 784, 10, Xt=Xt) for Wk in Ws[:3]]
    got = [f() for f in pending] + [K.eval_errors_async(Xc, yc, split, Wk.cuda(), 784, 10, Xt=Xt)() for Wk in Ws[3:]]
    for Wk, (a, b) in zip(Ws, got):
        ra = K.eval_error(X[:split], y[:split], Wk, 784, 10)
        rb = K.eval_error(X[split:], y[split:], Wk, 784, 10)
        assert abs(a - ra) <= 1.0 / split and abs(b - rb) <= 1.0 / (1000 - split)


@pytest.mark.parametrize("U1", [16, 23, 100])
def test_noise_gram_table_tiles_bit_identical(U1):
    """The noise-aware Gram with its noise x noise tiles copied from the setup table of the 100 periodic noise
    Grams (NoiseRows.gram_table) equals the Gram that computes them, bit for bit -- whole, and split over 3
    ranks' tile ranges -- for delta blocks that do and do not end on a tile boundary."""
    N, D = 37, 7850
    nr = K.NoiseRows(N, D, 11, "cuda")
    tab = nr.gram_table()
    assert tab.shape == (100, N, N) and torch.equal(tab[5], tab[5].T)
    g = torch.Generator().manual_seed(U1)
    X = (0.01 * torch.randn((U1, D), generator=g)).float().cuda()
    for it in (0, 5, 199):
        ref = K.gram_stacked_async(X, nr.rows(it))["gram"]
        got = K.gram_stacked_async(X, nr.rows(it), nn=tab[it % 100])["gram"]
        torch.cuda.synchronize()
        assert torch.equal(ref, got), (it, (ref - got).abs().max().item())
        parts = [K.gram_stacked_async(X, nr.rows(it), split=(r, 3), nn=tab[it % 100]) for r in range(3)]
        torch.cuda.synchronize()
        U = U1 + N
        _, _, chunk, npairs = K.gram_split(U, 0, 3)
        full = torch.cat([p["gram"][r * chunk:(r + 1) * chunk] for r, p in enumerate(parts)])[:npairs]
        assert torch.equal(ref, full)
    # the table's entries are the dense noise Gram (fp64 products of fp32 rows, summed exactly enough)
    rows = nr.rows(7).double()
    assert torch.allclose(tab[7], rows @ rows.T, rtol=1e-12, atol=1e-9)
