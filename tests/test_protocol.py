"""Protocol rules of the native runtime vs literal Python restatements of the reference logic."""
import pytest
import hashlib
import random

import numpy as np


def _ref_noisers(stake, n, inp, self_, nn):
    """DistSys/vrf.go:54-100 with the explicit ticket list."""
    tickets = [i for i in range(n) for _ in range(stake.get(i, 0))]
    res, seen, i, inp = [], set(), 0, bytes(inp)
    while len(res) < nn:
        if i + 1 >= len(inp):
            inp = hashlib.sha256(inp).digest()
            i = 0
        w = tickets[(inp[i] * 256 + inp[i + 1]) % len(tickets)]
        i += 1
        if w != self_ and w not in seen:
            seen.add(w)
            res.append(w)
    return res


def test_lottery_prefix_sums_match_ticket_list(rt):
    rnd = random.Random(1)
    for _ in range(200):
        n = rnd.randint(3, 60)
        stake = {i: rnd.choice([0, 10, 15, 500, 3]) for i in range(n)}
        stake.update({0: 10, 1: 7, 2: 9})
        out = bytes(rnd.getrandbits(8) for _ in range(64))
        s = rnd.randrange(n)
        assert list(rt.select_noisers(stake, out, s, 2, n)) == _ref_noisers(stake, n, out, s, 2)


def test_select_noisers_batch(rt):
    rnd = random.Random(2)
    stake = {i: 10 + 5 * rnd.randint(0, 400) for i in range(100)}
    outs = [bytes(rnd.getrandbits(8) for _ in range(64)) for _ in range(30)]
    selfs = list(range(30))
    got = rt.select_noisers_batch(stake, outs, selfs, 2, 100)
    assert [list(g) for g in got] == [list(rt.select_noisers(stake, o, s, 2, 100)) for o, s in zip(outs, selfs)]


def test_select_roles_distinct_and_stake_weighted(rt):
    stake = {i: 10 for i in range(20)}
    stake[7] = 100000
    hits = 0
    for k in range(50):
        v, m = rt.select_roles(stake, hashlib.sha256(bytes([k])).digest(), 3, 3, 20)
        assert len(set(v)) == 3 and len(set(m)) == 3
        hits += 7 in v
    assert hits == 50  # overwhelmingly staked peer is always drawn


def test_protocol_config_derivation(rt):
    pc = rt.ProtocolConfig()
    pc.num_nodes, pc.num_verifiers, pc.num_miners, pc.num_noisers = 100, 3, 3, 2
    pc.perc_samples, pc.poly_size, pc.poisoning, pc.colluders = 70, 10, 0.3, 0
    pc.derive()
    assert pc.num_samples == 70                    # int(N * ns / 100), <= N - nv - na
    assert pc.total_shares == 21                   # ceil(2 * poly / na) * na
    assert pc.shares_per_miner == 7
    assert pc.poisoning_index == 70                # ceil(N * (1 - po))


def test_gob_blockdata_hand_derived_vector(rt):
    """encoding/gob bytes of BlockData{Iteration: 3, GlobalW: [1.0], Deltas: [Update{SourceID: 2,
    Iteration: 3, Commitment: [0xAB], Accepted: true}]} as a fresh Go process's Encoder writes them
    (blockData.go:31-41), derived by hand from the encoding/gob wire spec -- not from our encoder.
    Go is not available here, so parity with real Go output stays unpinned; this pins the spec.

    Type ids: user ids start after firstUserId = 64 and are handed out while the type info is built:
    BlockData 65 (struct, id set before its fields), []float64 66, Update 67 (the element gets its
    id before the []Update slice does), [][]uint8 68, []main.Update 69.  Builtins: bool 1, int 2,
    float 4, []byte 5.  Ints are zig-zag (x<<1, negative: ^x<<1|1); uints >= 128 are a negated byte
    count then big-endian bytes; floats are the byte-reversed IEEE bits as a uint.  Messages are
    uint(length) + payload; type definitions go depth-first in field order, each before its inner
    types (Encoder.sendType), basic types and []byte are never described."""
    def s(txt):  # string field value: uint(len) + bytes
        return bytes([len(txt)]) + txt.encode()

    def field(name, tid):  # fieldType{Name, Id}: 01 name 01 id 00
        return b"\x01" + s(name) + b"\x01" + tid + b"\x00"

    ID65, ID66, ID67, ID68, ID69 = b"\xff\x82", b"\xff\x84", b"\xff\x86", b"\xff\x88", b"\xff\x8a"
    INT, FLOAT, BYTES, BOOL = b"\x04", b"\x08", b"\x0a", b"\x02"
    # 1. BlockData: -65, wireType.StructT (delta 3), structType.CommonType (delta 1){Name, Id}, Field (delta 1)
    m1 = (b"\xff\x81" + b"\x03" + b"\x01" + b"\x01" + s("BlockData") + b"\x01" + ID65 + b"\x00"
          + b"\x01" + b"\x03" + field("Iteration", INT) + field("GlobalW", ID66) + field("Deltas", ID69)
          + b"\x00" + b"\x00")
    # 2. []float64: -66, wireType.SliceT (delta 2), sliceType.CommonType, sliceType.Elem = float
    m2 = b"\xff\x83" + b"\x02" + b"\x01" + b"\x01" + s("[]float64") + b"\x01" + ID66 + b"\x00" + b"\x01" + FLOAT + \
        b"\x00" + b"\x00"
    # 3. []main.Update: -69, elem Update (67)
    m3 = b"\xff\x89" + b"\x02" + b"\x01" + b"\x01" + s("[]main.Update") + b"\x01" + ID69 + b"\x00" + b"\x01" + ID67 + \
        b"\x00" + b"\x00"
    # 4. Update: -67, eight fields
    m4 = (b"\xff\x85" + b"\x03" + b"\x01" + b"\x01" + s("Update") + b"\x01" + ID67 + b"\x00" + b"\x01" + b"\x08"
          + field("SourceID", INT) + field("Iteration", INT) + field("Delta", ID66) + field("Commitment", BYTES)
          + field("Noise", ID66) + field("NoisedDelta", ID66) + field("Accepted", BOOL)
          + field("SignatureList", ID68) + b"\x00" + b"\x00")
    # 5. [][]uint8: -68, elem []byte (5)
    m5 = b"\xff\x87" + b"\x02" + b"\x01" + b"\x01" + s("[][]uint8") + b"\x01" + ID68 + b"\x00" + b"\x01" + BYTES + \
        b"\x00" + b"\x00"
    # 6. the value: type id 65, then the non-zero fields as (field-number delta, value), 0 terminator
    upd = (b"\x01" + b"\x04"              # SourceID (field 0): int 2
           + b"\x01" + b"\x06"            # Iteration (1): int 3
           + b"\x02" + b"\x01\xab"        # Commitment (3, delta 2): []byte len 1, 0xAB
           + b"\x03" + b"\x01"            # Accepted (6, delta 3): true
           + b"\x00")
    m6 = (ID65 + b"\x01" + b"\x06"        # Iteration (0): int 3
          + b"\x01" + b"\x01" + b"\xfe\xf0\x3f"  # GlobalW (1): 1 element, 1.0 = bits 3ff0... reversed -> 0xf03f
          + b"\x01" + b"\x01" + upd       # Deltas (2): 1 element
          + b"\x00")

    def msg(p):
        n = len(p)
        return (bytes([n]) if n < 128 else b"\xff" + bytes([n])) + p
    expect = b"".join(msg(m) for m in (m1, m2, m3, m4, m5, m6))
    assert [len(m) for m in (m1, m2, m3, m4, m5, m6)] == [62, 23, 28, 133, 23, 22]
    d = rt.BlockData()
    d.iteration = 3
    d.global_w = [1.0]
    u = rt.Update()
    u.source_id, u.iteration, u.commitment, u.accepted = 2, 3, b"\xab", True
    d.deltas = [u]
    assert bytes(d.gob()) == expect


def test_runconfig_rejects_unsupported_shapes():
    import pytest as _pt

    from biscotti_amd.protocol.config import RunConfig

    RunConfig(num_nodes=200).validate()               # 200 peers: inbox 140
    RunConfig(num_nodes=400).validate()               # inbox 280 > 256: the sorted-row Krum kernels
    RunConfig(num_nodes=100, dataset="lfw").validate()
    for bad in (dict(num_nodes=6000), dict(num_verifiers=65, num_nodes=200), dict(num_miners=1, poly_size=20),
                dict(batch_size=32), dict(dataset="cifar"), dict(num_nodes=5, num_verifiers=3, num_miners=2)):
        with _pt.raises(ValueError):
            RunConfig(**bad).validate()


def test_gob_float_vector_matches_scalar_encoder(rt):
    """The block's model vector goes through the raw-pointer vector encoder: its bytes equal the
    per-value gob float encoding (byte-reversed IEEE bits as a uint) for edge values and random ones."""
    import struct

    import numpy as np

    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 2.0 ** -1074, 1e308, -1e-300, float("inf"), float("-inf"), 3.0, 1.0 / 3]
    vals += np.random.default_rng(5).standard_normal(500).tolist()
    d = rt.BlockData()
    d.global_w = vals
    enc = d.gob()
    body = b"".join(rt.gob_float(v) for v in vals)
    assert body in enc

    def slow(v):   # the wire spec, in Python
        rev = int.from_bytes(struct.pack("<d", v), "big")
        if rev < 128:
            return bytes([rev])
        raw = rev.to_bytes(8, "big").lstrip(b"\x00")
        return bytes([256 - len(raw)]) + raw
    assert all(rt.gob_float(v) == slow(v) for v in vals)


def test_select_noisers_job_matches_per_worker_lottery():
    """The batched noiser draw that reads a VRF batch's outputs natively (one ticket table for every
    worker, output index remapping) equals select_noisers run per worker on the same outputs."""
    from biscotti_amd.native import rt

    R = rt()
    stake = {i: 10 + (i * 7) % 50 for i in range(60) if i % 9}
    seeds = [bytes([i]) * 32 for i in range(60)]
    job = R.vrf_prove_batch_async(seeds, b"alpha" * 6 + b"xy", 2, None, True)
    betas = job.betas()
    selfs = list(range(5, 55))
    idx = [s for s in selfs]
    for nn in (1, 2, 3):
        got = R.select_noisers_job(stake, job, idx, selfs, nn, 60).tolist()
        assert got == [R.select_noisers(stake, betas[i], s, nn, 60) for i, s in zip(idx, selfs)]
    assert R.select_noisers_job(stake, job, [], list(range(60)), 2, 60).tolist() == \
        R.select_noisers_batch(stake, betas, list(range(60)), 2, 60)


def test_select_noisers_after_block_uses_the_stake_it_leaves():
    """The speculative front's noiser lottery (select_noisers_job_after) draws with the stake the block leaves the
    FSM with once committed: the block's own map, or the FSM's when the block carries none."""
    from biscotti_amd.native import rt
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    R = rt()
    eng = BiscottiEngine(RunConfig(num_nodes=12, dataset="mnist", seed=5, max_iterations=100,
                                   deterministic_time=True), Comm())
    eng.run_round()
    fsm, blk = eng.fsm, eng.fsm.chain.latest()
    job = R.vrf_prove_batch_async([bytes([i]) * 32 for i in range(12)], bytes(blk.hash), 2, None, True)
    ws = list(range(12))
    other = {i: 1 + 5 * i for i in range(12)}
    assert other != dict(fsm.stake)
    blk.stake = other
    got = R.select_noisers_job_after(fsm, blk, job, [], ws, 2, 12).tolist()
    assert got == R.select_noisers_job(other, job, [], ws, 2, 12).tolist()
    blk.stake = {}
    got = R.select_noisers_job_after(fsm, blk, job, [], ws, 2, 12).tolist()
    assert got == fsm.select_noisers_job(job, [], ws, 2, 12).tolist()
    eng.close()


def test_successor_gives_the_next_plan_before_commit():
    """fsm.successor(block) (used to launch the next round's share MSM before the block's audit is read)
    yields the same plan, verifier inboxes and leader arrival order as the FSM after the commit."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    eng = BiscottiEngine(RunConfig(num_nodes=12, dataset="mnist", seed=7, max_iterations=100,
                                   deterministic_time=True), Comm())
    for _ in range(3):
        eng.run_round()
        fsm = eng.fsm
        live = [1] * 12
        shadow = fsm.successor(fsm.chain.latest())
        p1 = shadow.begin_round(live)
        got = (list(p1.verifiers), list(p1.miners), list(p1.workers), p1.iteration,
               [list(x) for x in shadow.verifier_inboxes(list(p1.workers))], list(shadow.leader_arrivals()))
        saved = fsm.iteration
        p2 = fsm.begin_round(live)
        want = (list(p2.verifiers), list(p2.miners), list(p2.workers), p2.iteration,
                [list(x) for x in fsm.verifier_inboxes(list(p2.workers))], list(fsm.leader_arrivals()))
        fsm.iteration = saved   # undo the probe's begin_round
        assert got == want
    eng.close()


@pytest.mark.parametrize("nv,lo,hi", [(3, 0, 12), (3, 4, 9), (1, 0, 12), (1, 2, 7)])
def test_spec_plan_matches_python_composition(nv, lo, hi):
    """RoundFSM.spec_plan (the next round's speculative plan in one native call) == the composition of
    successor / begin_round / verifier_inboxes / leader_arrivals it replaces, candidates included (the
    floor(nv/2) == 0 case takes every worker)."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    eng = BiscottiEngine(RunConfig(num_nodes=12, dataset="mnist", seed=3, max_iterations=100, num_verifiers=nv,
                                   deterministic_time=True), Comm())
    for _ in range(3):
        eng.run_round()
        blk = eng.fsm.chain.latest()
        shadow = eng.fsm.successor(blk)
        p = shadow.begin_round([1] * 12)
        workers = list(p.workers)
        ibs = [list(x) for x in shadow.verifier_inboxes(workers)]
        cand = set(workers) if len(p.verifiers) // 2 == 0 else set().union(*ibs)
        arr = list(shadow.leader_arrivals())
        rank = {w: i for i, w in enumerate(arr)}
        spec = sorted((w for w in workers if lo <= w < hi and w in cand), key=lambda w: rank.get(w, 1 << 30))
        plan, ibs2, arr2, spec2, cands2, order2 = eng.fsm.spec_plan(blk, lo, hi)
        order = [w for w in arr if w in cand]
        assert list(order2) == order
        assert (list(plan.verifiers), list(plan.miners), list(plan.workers), plan.iteration) == \
            (list(p.verifiers), list(p.miners), workers, p.iteration)
        assert [list(x) for x in ibs2] == ibs and list(arr2) == arr and list(spec2) == spec
        assert list(cands2) == sorted(cand)
        # Krum's static tables (verify.py _krum_static) for a non-identity peer -> row mapping
        xrow = {q: (11 - q) for q in range(12) if q % 5}
        xl = [xrow.get(q, -1) for q in range(12)]
        got = eng.fsm.spec_plan(blk, lo, hi, xl, 12)
        np.testing.assert_array_equal(got[5], np.array([[xl[w] for w in ib] for ib in ibs], np.int32).reshape(len(ibs), -1))
        want_rank = np.full(12, -1, np.int32)
        for i, w in enumerate(arr):
            if xl[w] >= 0:
                want_rank[xl[w]] = i
        np.testing.assert_array_equal(got[6], want_rank)
        np.testing.assert_array_equal(got[7], np.array([xl[w] for w in spec], np.int32))
        # a horizon keeps the first h candidates in the leader's arrival order (head.py SPEC_MARGIN)
        h = max(1, len(order) // 2)
        gh = eng.fsm.spec_plan(blk, lo, hi, xl, 12, h)
        keep = set(order[:h])
        spec_h = [w for w in spec if w in keep]
        assert list(gh[3]) == spec_h and list(gh[4]) == sorted(keep) and list(gh[8]) == order
        np.testing.assert_array_equal(gh[7], np.array([xl[w] for w in spec_h], np.int32))
    eng.close()


def test_cli_defaults_match_runconfig():
    """The reference + framework flags with an empty argv give RunConfig() exactly (no knob whose CLI
    default silently differs from the config default, e.g. a store_false flag turning phase sync on);
    --fail-at/--fail-rank and --no-roles-vrf-proof map onto fail_at / ablation."""
    import argparse

    from biscotti_amd.protocol.config import RunConfig, add_framework_flags, add_reference_flags, config_from_args

    ap = argparse.ArgumentParser()
    add_reference_flags(ap)
    add_framework_flags(ap)
    assert config_from_args(ap.parse_args([])) == RunConfig()
    cfg = config_from_args(ap.parse_args(["--fail-at", "2", "--fail-rank", "1", "--no-roles-vrf-proof",
                                          "--phase-sync"]))
    assert cfg.fail_point() == (2, 1) and not cfg.roles_vrf_proof and cfg.phase_sync
    assert RunConfig().fail_point() == (-1, 0)
    import dataclasses

    # 49 + phase_log (the reference's phase lines, round 5) + miner_threshold (main.go:348-360, round 6)
    assert len(dataclasses.fields(RunConfig)) <= 51
    import pytest

    with pytest.raises(ValueError):
        RunConfig(ablation="early_krum").validate()


def test_route_view_matches_route_shares_and_leader_view():
    """RoundFSM.route_view (share routing + the leader's view in one native call) == route_shares followed
    by leader_view and the first node's share part per contributing miner, with all miners live and with
    one miner offline."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    eng = BiscottiEngine(RunConfig(num_nodes=14, dataset="mnist", seed=4, max_iterations=100,
                                   deterministic_time=True), Comm())
    eng.run_round()
    fsm = eng.fsm
    for kill in (None, 0):
        live = [1] * 14
        plan = fsm.begin_round(live)
        if kill is not None:
            live[list(plan.miners)[kill]] = 0
            plan = fsm.begin_round(live)
        approved = list(plan.workers)[: 7]
        routes = fsm.route_shares(approved)
        lv = fsm.leader_view(routes)
        online, quorum, nodes, contrib, part = fsm.route_view(approved)
        assert (online, quorum, list(nodes), list(contrib)) == \
            (lv.leader_online, lv.quorum, list(lv.node_list), list(lv.contributing_miners))
        if nodes:
            assert part == {m: dict(routes[m])[nodes[0]] for m in contrib}
        fsm.iteration -= 1   # undo the probe's begin_round
    eng.close()


def test_spec_horizon_policy():
    """head.py's speculative horizon: every candidate (-1) until SPEC_MIN_HISTORY blocks are known, then the
    leader's cap + SPEC_MARGIN or the deepest recent block row + SPEC_SLACK (+2 per missing window block),
    whichever is further; block depths are kept for the last SPEC_WINDOW blocks."""
    from types import SimpleNamespace

    from biscotti_amd.protocol import head as H

    class Cfg:
        def __init__(self, abl=""):
            self.abl = abl

        def has(self, a):
            return a == self.abl

    eng = SimpleNamespace(fsm=SimpleNamespace(leader_cap_size=lambda: 35), cfg=Cfg())
    horizon = H.RoundHeadMixin._spec_horizon
    note = H.RoundHeadMixin._note_block_depth
    assert horizon(eng) == -1
    order = list(range(100, 194))   # candidates in leader arrival order
    for depth in (40, 44, 38):
        note(eng, {"cand_order": order}, [order[depth - 1], order[3]])
    assert eng._spec_depths == [40, 44, 38]
    # 3 of 8 window blocks known: max(35 + 16, 44 + 8 + 2 * 5)
    assert horizon(eng) == max(35 + H.SPEC_MARGIN, 44 + H.SPEC_SLACK + 2 * (H.SPEC_WINDOW - 3)) == 62
    for _ in range(10):
        note(eng, {"cand_order": order}, [order[29]])
    assert len(eng._spec_depths) == H.SPEC_WINDOW and horizon(eng) == 35 + H.SPEC_MARGIN
    note(eng, {"cand_order": order}, [order[79]])   # a deep block widens the next horizons
    assert horizon(eng) == 80 + H.SPEC_SLACK
    eng.cfg = Cfg("spec_all_candidates")
    assert horizon(eng) == -1
    eng.cfg = Cfg("spec_tight")
    assert horizon(eng) == 35
    eng.cfg, eng.fsm = Cfg(), SimpleNamespace(leader_cap_size=lambda: 0)   # no leader cap: every candidate
    assert horizon(eng) == -1


@pytest.mark.parametrize("rule,n,want", [("half_samples", 100, 35), ("eighth", 100, 12), ("eighth", 50, 6),
                                         ("eighth", 12, 2), ("tenth", 50, 5), ("tenth", 14, 2)])
def test_miner_threshold_rules(rt, rule, n, want):
    """The leader miner's block size: NUM_SAMPLES/2 (main.go:360), numberOfNodes/8 (minBlockSize,
    main.go:348-352) or /10 (what nsdi-eval/churn/*.log fired at: 'I expect 5 shares' with 50 peers), floor 2."""
    from biscotti_amd.protocol.config import RunConfig

    cfg = RunConfig(num_nodes=n, miner_threshold=rule)
    cfg.validate()
    pc = cfg.protocol(rt)
    assert pc.miner_share_thresh == want
    # the plain path's leader keeps NUM_SAMPLES/2 updates (processUpdate, main.go:1222-1230)
    import dataclasses

    assert dataclasses.replace(cfg, secure_agg=False).protocol(rt).miner_share_thresh == pc.num_samples // 2


def test_runconfig_rejects_unknown_miner_threshold():
    from biscotti_amd.protocol.config import RunConfig

    with pytest.raises(ValueError, match="miner_threshold"):
        RunConfig(miner_threshold="quarter").validate()


def test_leader_fires_at_an_eighth_of_the_nodes():
    """Secure rounds with miner_threshold=eighth: every non-empty block carries exactly floor(N/8) updates (the
    leader's first arrivals among the approved; the approved always outnumber it here), the chain verifies and
    the stake grows by stake_unit per contributor."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    n = 24
    eng = BiscottiEngine(RunConfig(num_nodes=n, dataset="mnist", seed=3, max_iterations=100, deterministic_time=True,
                                   miner_threshold="eighth", device="cpu"), Comm())
    assert eng.fsm.leader_cap_size() == n // 8
    stake0 = sum(dict(eng.fsm.stake).values())
    sizes = []
    for _ in range(3):
        r = eng.run_round()
        if not r.empty:
            sizes.append(len(r.node_list))
            assert len(r.approved) > n // 8
    assert sizes and all(s == n // 8 for s in sizes), sizes
    assert sum(dict(eng.fsm.stake).values()) == stake0 + 5 * sum(sizes)
    ok, why = eng.fsm.chain.verify()
    assert ok, why
    eng.close()
