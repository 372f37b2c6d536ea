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
    if eng._native is not None:
        # the pre-step runs natively (NativeSecAgg.prestep / after_select): record its quantised updates too
        pre_fn = eng._native._pre_out

        def pre_spy(k, W, it):
            out = pre_fn(k, W, it)
            torch.cuda.current_stream().wait_event(out["ev"])   # the step runs on the Gram stream
            seen.update({(it, p): out["qdelta"][i].clone() for i, p in enumerate(eng.task.peers)})
            return out
        eng._native._pre_out = pre_spy
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


def test_heavy_churn_without_miner_quorum():
    """Rounds where too few miners are live for a quorum (shares_per_miner x live miners < POLY_SIZE)
    end in empty blocks; the device-side aggregation is not queued for them (it would have fewer
    share points than coefficients)."""
    eng = _engine(num_nodes=20, churn=0.6)
    res = _run_exact(eng, 25)
    assert len(res) == 25 and any(r.empty for r in res) and any(not r.empty for r in res)
    assert eng.fsm.chain.verify()[0]


def test_poisoners_on_gpu():
    eng = _engine(num_nodes=20, poisoning=0.3)
    pois = {p for p in range(20) if eng.fsm.is_poisoner(p)}
    assert pois
    res = _run_exact(eng, 5)
    assert all(set(r.node_list) <= set(r.approved) for r in res)


@pytest.mark.parametrize("nv,extra", [(3, {"ablation": "noise_independent"}), (5, {"ablation": "noise_independent"}),
                                      (3, {"noising": False})])
def test_krum_rejects_label_flip_poisoners(nv, extra):
    """30% 1->7 label-flip poisoners, every verifier with its own inbox: after a 10-round burn-in at
    least 90% of the poisoners' updates that reach a verifier stay out of the blocks.  Run with
    per-worker DP noise (ablation) or without noise: with the reference's shared pre-sampled noiser
    vectors the noise-sharing structure, not the gradients, dominates Krum's distances on the
    synthetic digits (docs/ROBUSTNESS.md; profiles/poison_r2*.json)."""
    eng = _engine(num_nodes=50, poisoning=0.3, num_verifiers=nv, epsilon=1.0, **extra)
    pois = {p for p in range(50) if eng.fsm.is_poisoner(p)}
    seen = kept = 0
    for _ in range(20):
        r = eng.run_round()
        if r.iteration < 10:
            continue
        judged = set().union(*r.inboxes.values()) if r.inboxes else set()
        seen += len(judged & pois)
        kept += len(set(r.node_list) & pois)
    ok, why = eng.fsm.chain.verify()
    eng.close()
    assert ok, why
    assert seen > 0
    assert kept <= 0.1 * seen, (kept, seen)


def test_single_verifier_quirk_aggregates_rejected_updates():
    """nv = 1: floor(1/2) = 0 signatures approve every live worker, including updates the verifier's
    Krum rejected (main.go:1686) -- their shares must be computed, not cancelled (blocks stay
    non-empty and exact)."""
    eng = _engine(num_nodes=12, num_verifiers=1, num_miners=3)
    res = _run_exact(eng, 4)
    assert all(not r.empty for r in res)
    assert any(set(r.node_list) - set(r.approved_by_krum) for r in res)


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


@pytest.mark.parametrize("noising", [True, False])
def test_deferred_signatures_valid_on_gpu(noising):
    """GPU secure path: the verifiers' signature batch starts behind the next round's VRF outputs and
    is joined a round later; after drain() every accepted slot verifies against the worker's
    commitment in the block, and an uninterrupted run keeps its chain valid."""
    eng = _engine(num_nodes=20, num_verifiers=3, noising=noising)
    for _ in range(4):
        r = eng.run_round()
        eng.drain()
        sig = eng.last_signatures
        blk = eng.fsm.chain.latest()
        commits = {w: bytes(u.commitment) for w, u in zip(r.node_list, blk.data.deltas)} if not r.empty else {}
        n_ok = 0
        for vi, v in enumerate(r.verifiers):
            for j, w in enumerate(r.inboxes.get(v, [])):
                s_ = sig[vi, j].tobytes()
                if any(s_) and w in commits:
                    assert eng.R.schnorr_verify(commits[w], eng.pk[v], s_)
                    n_ok += 1
        assert r.empty or n_ok > 0
    for _ in range(4):   # rounds without drain: each joins the previous round's batch
        eng.run_round()
    eng.drain()
    assert eng.fsm.chain.verify()[0]
    assert eng.stats.get("early_vrf", 0) >= 6 and eng.stats.get("device_aggregations", 0) >= 6
    eng.close()


def test_lazy_eval_resolves_the_same_numbers():
    """lazy_eval (bench.py): a round's test error / attack rate are read back in the next round or by
    drain(); they equal the eagerly read numbers of the same deterministic run."""
    out = []
    for lazy in (False, True):
        eng = _engine(num_nodes=16, lazy_eval=lazy)
        rs = [eng.run_round() for _ in range(4)]
        eng.drain()
        out.append([(r.iteration, r.test_error, r.attack_rate) for r in rs])
        eng.close()
    assert out[0] == out[1]
    assert all(e == e for _, e, _ in out[1])   # no NaN left after drain()


def test_mnist_label_flip_rejection_floor_default_noise():
    """BASELINE config 4 (MNIST, 30% 1->7 label-flip poisoners, epsilon 1) under the reference's DEFAULT
    noise semantics (workers noised with their noisers' shared pre-sampled vectors, client_obj.py:97-98):
    after a 10-round burn-in at least 75% of the poisoners' updates that reach a verifier stay out of the
    blocks -- today's measured floor (0.80-0.84 rejection at 100 peers, docs/ROBUSTNESS.md), asserted so a
    regression shows.  The reference's 0.029 attack rate stays parity-unpinned (synthetic digits)."""
    eng = _engine(num_nodes=100, poisoning=0.3, epsilon=1.0, seed=7)
    pois = {p for p in range(100) if eng.fsm.is_poisoner(p)}
    seen = kept = 0
    attack = []
    for _ in range(30):
        r = eng.run_round()
        attack.append(r.attack_rate)
        if r.iteration < 10:
            continue
        judged = set().union(*r.inboxes.values()) if r.inboxes else set()
        seen += len(judged & pois)
        kept += len(set(r.node_list) & pois)
    ok, why = eng.fsm.chain.verify()
    eng.close()
    assert ok, why
    assert seen > 0
    assert kept <= 0.25 * seen, (kept, seen)
    # the attack's effect (get17AttackRate: digit-1 error) over rounds 20-29, next to the rejection floor
    last10 = sum(attack[-10:]) / 10
    print("digit-1 error, rounds 20-29:", round(last10, 4), "rejection", round(1 - kept / seen, 4))
    assert last10 <= DIGIT1_ERR_CEILING, last10


# this deterministic run measures 0.647 (rejection 0.756); the reproducible 5-seed poison30 run (bench.py
# --deterministic-time --seeds 5, round 6) gives 0.582 +- 0.065 with a worst seed of 0.644: ceiling 0.70
DIGIT1_ERR_CEILING = 0.70


@pytest.mark.parametrize("poisoning", [0.0, 0.3])
def test_spec_horizon_same_chain_as_every_candidate(poisoning):
    """The speculative share MSM covers the leader's candidate arrivals up to an adaptive horizon (head.py
    SPEC_MARGIN) instead of every candidate: the chain is byte-identical to computing every candidate's shares
    (ablation spec_all_candidates) -- blocks reaching past the horizon are topped up by the host path -- and it
    launches fewer rows.  spec_tight (horizon = the leader's cap) makes the host top-up path frequent: same chain."""
    out = []
    for abl in ("", "spec_all_candidates", "spec_tight"):
        eng = _engine(num_nodes=100, poisoning=poisoning, epsilon=1.0, seed=11, ablation=abl)
        hashes = [bytes(eng.run_round().block_hash) for _ in range(8)]   # the horizon applies after 3 blocks
        rows8 = eng.stats.get("spec_rows", 0)
        hashes += [bytes(eng.run_round().block_hash) for _ in range(6)]
        eng.stats["spec_rows_late"] = eng.stats.get("spec_rows", 0) - rows8
        eng.drain()
        ok, why = eng.fsm.chain.verify()
        stats = dict(eng.stats)
        eng.close()
        assert ok, why
        out.append((hashes, stats))
    (h0, s0), (h1, s1), (h2, s2) = out
    assert h0 == h1 == h2
    if poisoning:
        assert s2.get("spec_misses", 0) > 0, s2   # rejections among the first cap arrivals: the host path ran
        # ... topping the speculative slot up with the missing rows (not recomputing every block row)
        assert s2.get("spec_topups", 0) == s2["spec_misses"], s2
    assert s0.get("spec_head", 0) >= 6 and s1.get("spec_head", 0) >= 6
    assert s0["spec_rows_late"] < 0.9 * s1["spec_rows_late"], (s0["spec_rows_late"], s1["spec_rows_late"])
    print("rows launched after the window", s0["spec_rows_late"], "vs", s1["spec_rows_late"], "misses",
          s0.get("spec_misses", 0), "tight misses", s2.get("spec_misses", 0))


def test_close_after_plain_rounds_with_a_pending_front():
    """run_round() without last=True leaves the next round's front launched (its Krum, the aggregation queued
    behind it, a suspended verification generator, unjoined VRF jobs): close() must stop and drop it before it
    releases the streams, and a second engine must run normally afterwards."""
    eng = _engine(num_nodes=30, lazy_eval=True)
    for _ in range(4):
        eng.run_round()
    assert eng._front is not None and eng.stats.get("early_fronts", 0) >= 2
    eng.close()
    assert eng._front is None
    eng2 = _engine(num_nodes=30)
    r = eng2.run_round()
    assert not r.empty and eng2.fsm.chain.verify()[0]
    eng2.close()


def test_lagging_evaluation_reads_its_own_model():
    """The evaluation runs on the low-priority witness stream and may lag the main stream by several rounds,
    while the native W ring slot it was given is rewritten by later recoveries: with the witness stream stalled
    (a long sleep kernel queued on it every round) the reported test errors equal an unstalled run's."""
    out = []
    for stall in (False, True):
        eng = _engine(num_nodes=30, lazy_eval=True)
        errs = []
        for k in range(8):
            if stall:
                with torch.cuda.stream(eng.witness_stream):
                    torch.cuda._sleep(20_000_000)   # ~10 ms of the witness stream per round
            errs.append(eng.run_round(last=k == 7))
        eng.drain()
        out.append([(r.iteration, r.test_error, r.attack_rate) for r in errs])
        eng.close()
    assert out[0] == out[1]
    assert all(e == e for _, e, _ in out[1])


def test_audit_read_back_is_per_audit():
    """Two aggregate audits queued before either is read (the speculative front queues the next round's before the
    current one's verdicts are read) each read back their own verdicts: the first over the last round's consistent
    coefficients passes, the second over tampered ones fails one chunk."""
    eng = _engine()
    for _ in range(3):
        eng.run_round()
    eng.drain()
    torch.cuda.synchronize()
    na = eng._native
    assert na is not None
    first = na.audit(queue=True)
    na.coeffs[0, 0] += 1   # stream-ordered after the first audit's read of the coefficients
    second = na.audit(queue=True)
    bad = second().copy()
    good = first().copy()
    assert good.all(), good
    assert bad[0, 0] == 0 and bad.sum() == bad.size - 1, bad
    na.coeffs[0, 0] -= 1
    eng.close()
