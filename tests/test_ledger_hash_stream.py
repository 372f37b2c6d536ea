"""The streaming block hash (ledger.cpp Block::compute_hash: GlobalW gob-encoded straight into SHA-256 in
pieces, the message length from a length pass) equals sha256(prev_hash || timestamp || gob(data)) over the
materialised gob (block.go:27-35 setHash) for every BlockData shape."""
import hashlib

import numpy as np
import pytest

from biscotti_amd.native import rt


def _expected(b) -> bytes:
    return hashlib.sha256(bytes(b.prev_hash) + str(b.timestamp).encode() + bytes(b.data.gob())).digest()


@pytest.mark.parametrize("nw", [0, 1, 447, 448, 449, 7850])
@pytest.mark.parametrize("nd", [0, 3])
@pytest.mark.parametrize("it", [-1, 0, 7])
def test_stream_hash_matches_gob(nw, nd, it):
    R = rt()
    rng = np.random.default_rng(nw * 31 + nd * 7 + it + 1)
    b = R.Block()
    b.timestamp = 0 if nd == 0 else 1700000000 + nw
    b.prev_hash = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    d = R.BlockData()
    d.iteration = it
    # values spanning every gob float length: zeros, small integers, +-1e-300..1e300, negative zero
    w = rng.standard_normal(nw) * 10.0 ** rng.integers(-300, 300, nw)
    if nw:
        w[:: max(1, nw // 5)] = 0.0
        w[1:: max(2, nw // 3)] = 2.0
        w[-1] = -0.0
    d.global_w = w
    ups = []
    for k in range(nd):
        u = R.Update()
        u.source_id, u.iteration, u.accepted = k, it, bool(k % 2)
        u.commitment = bytes(rng.integers(0, 256, 64, dtype=np.uint8))
        u.delta = list(rng.standard_normal(5)) if k == 1 else []
        u.signatures = [bytes(70), bytes(71)] if k == 2 else []
        ups.append(u)
    d.deltas = ups
    b.data = d
    assert bytes(b.compute_hash()) == _expected(b)


def test_secagg_block_hash_matches_gob():
    from biscotti_amd.protocol.config import RunConfig

    R = rt()
    cfg = RunConfig(dataset="mnist", num_nodes=20)
    fsm = R.RoundFSM(cfg.protocol(R), 7850)
    fsm.begin_round([1] * 20)
    W = np.random.default_rng(3).standard_normal(7850)
    nodes = [3, 5, 8]
    b = fsm.make_secagg_block(W, nodes, [bytes([k]) * 64 for k in range(3)], 12345)
    assert bytes(b.hash) == _expected(b)
    assert np.array_equal(np.asarray(b.data.global_w), W) and b.data.n_deltas == 3
    e = fsm.make_secagg_block(W, [], [], 12345)   # empty block: the latest block's W, timestamp 0
    assert bytes(e.hash) == _expected(e) and e.timestamp == 0 and not np.any(np.asarray(e.data.global_w))


def test_secagg_block_from_jacobian_rows():
    """make_secagg_block_jac (the block's commitments marshalled natively from the pre-step's device-layout
    Jacobian rows) builds the same block as make_secagg_block with the marshals g1_marshal_jac_batch gives."""
    from biscotti_amd.protocol.config import RunConfig

    R = rt()
    one = np.array([0xa1f76999, 0xe7a35393, 0xdf4a4a61, 0x11a4772e, 0x9e7b23de, 0x55901347, 0xb55c7806, 0x704afe1c],
                   np.uint32)   # Montgomery 1 (bn256_dev.h ONE): Z of an affine point in Jacobian form
    pts = [R.g1_base_mul(k * 7919 + 3) for k in range(12)]
    jac = np.stack([np.concatenate([np.asarray(R.g1_affine_mont_u32(p), np.uint32).reshape(-1)[:16], one])
                    for p in pts])
    jac[5] = 0   # the point at infinity (Z = 0)
    ref = R.g1_marshal_jac_batch(jac)
    assert bytes(ref[0]) == bytes(pts[0]) and not np.any(ref[5])
    cfg = RunConfig(dataset="mnist", num_nodes=20)
    fsm = R.RoundFSM(cfg.protocol(R), 7850)
    fsm.begin_round([1] * 20)
    W = np.random.default_rng(5).standard_normal(7850)
    nodes, rows = [2, 4, 9, 11], [7, 0, 5, 11]
    a = fsm.make_secagg_block_jac(W, nodes, jac, rows, 777)
    b = fsm.make_secagg_block(W, nodes, [bytes(ref[r]) for r in rows], 777)
    assert bytes(a.hash) == bytes(b.hash) == _expected(a)
    assert [bytes(u.commitment) for u in a.data.deltas] == [bytes(ref[r]) for r in rows]
