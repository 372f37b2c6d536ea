"""Protocol rules of the native runtime vs literal Python restatements of the reference logic."""
import hashlib
import random


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
