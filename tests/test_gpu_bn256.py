"""Numerics of the gfx950 BN256 kernels against the host runtime / Python big integers."""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
R = 1 << 256
RINV = pow(R, -1, P)


def _limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def _from_limbs(row):
    return sum(int(v) << (32 * i) for i, v in enumerate(row))


def _to_dev(vals):
    a = np.array([_limbs(v) for v in vals], dtype=np.uint32)
    return torch.from_numpy(a.view(np.int32)).cuda()


def _from_dev(t):
    a = t.cpu().numpy().view(np.uint32)
    return [_from_limbs(r) for r in a]


def test_field_ops_match_bigint():
    from biscotti_amd.ops import bn256 as B
    rnd = random.Random(3)
    xs = [0, 1, P - 1, P - 2, (1 << 255), R % P] + [rnd.randrange(P) for _ in range(2000)]
    ys = [P - 1, 1, P - 1, 3, (1 << 255) - 1, 7] + [rnd.randrange(P) for _ in range(2000)]
    a, b = _to_dev(xs), _to_dev(ys)
    assert _from_dev(B.fp_op(a, b, 0)) == [(x * y * RINV) % P for x, y in zip(xs, ys)]
    assert _from_dev(B.fp_op(a, b, 1)) == [(x + y) % P for x, y in zip(xs, ys)]
    assert _from_dev(B.fp_op(a, b, 2)) == [(x - y) % P for x, y in zip(xs, ys)]
    # Montgomery inverse: inv(xR) = x^-1 R  -> fp_inv works on the raw value: a^(p-2) in Montgomery domain
    got = _from_dev(B.fp_op(a, b, 3))
    for x, g in zip(xs[:200], got[:200]):
        assert g == (pow(x * RINV, P - 2, P) * R) % P
    assert _from_dev(B.fp_op(a, b, 4)) == [(x * RINV) % P for x in xs]


def _aff_dev(rt, pts):
    arr = np.concatenate([rt.g1_affine_mont_u32(p) for p in pts], axis=0)
    return torch.from_numpy(arr.view(np.int32)).cuda()


def test_point_ops_match_host(rt):
    from biscotti_amd.ops import bn256 as B
    g = rt.g1_generator()
    rnd = random.Random(5)
    ks_a = [rnd.randrange(1, 1 << 200) for _ in range(64)] + [5, 5, 7]
    ks_b = [rnd.randrange(1, 1 << 200) for _ in range(64)] + [10, 0, 0]
    A = [rt.g1_mul(g, k) for k in ks_a]
    Bp = [rt.g1_mul(g, k) for k in ks_b]
    a, b = _aff_dev(rt, A), _aff_dev(rt, Bp)
    small = torch.tensor([rnd.randrange(-1000, 1000) for _ in A], dtype=torch.int32, device="cuda")
    order = rt.bn256_order()
    for op in range(4):
        out = B.marshal(B.point_op(a, b, small, op)).cpu().numpy()
        for i, (ka, kb) in enumerate(zip(ks_a, ks_b)):
            if op in (0, 1):
                k = 2 * ka + kb
            elif op == 2:
                k = 2 * ka
            else:
                k = ka * int(small[i]) % order
            assert bytes(out[i]) == rt.g1_mul(g, k % order), (op, i)


@pytest.mark.parametrize("d,secret,scale,b0", [(25, 2, 10**4, 8), (57, 2, 10**6, 14), (33, 987654321123, 10**12, 11),
                                                (40, 2, 2**62, 14), (40, 2, 2**62, 8), (31, 7, 9000, 14)])
def test_shares_msm_matches_host(rt, d, secret, scale, b0):
    from biscotti_amd.ops import bn256 as B
    key = rt.CommitKey.generate(d, secret)
    eng = B.DeviceCommitEngine(key, poly=10, total_shares=21, b0=b0)
    rng = np.random.default_rng(d)
    P_ = 3
    coeffs = rng.integers(-scale, scale, size=(P_, d), dtype=np.int64)
    coeffs[0, :7] = 0                     # zero scalars
    coeffs[1, 3] = 2; coeffs[1, 4] = 1    # collisions with 2^i keys exercise doubling / P == -Q
    coeffs[2, :] = rng.integers(-3, 3, size=d)
    ct = torch.from_numpy(coeffs).cuda()
    rows = torch.tensor([2, 0, 1], dtype=torch.int32, device="cuda")
    pts, ys = eng.shares(ct, rows)
    comm = B.marshal(eng.commitments(pts)).cpu().numpy()
    allb = B.marshal(pts).cpu().numpy().reshape(3, eng.nchunks, 22, 64)
    ys = ys.cpu().numpy()
    for r, row in enumerate([2, 0, 1]):
        commitment, chunk_commits, hys, wits = key.make_shares(coeffs[row], 10, 21)
        assert bytes(comm[r]) == commitment
        assert bytes(comm[r]) == key.commit(coeffs[row], 0)
        np.testing.assert_array_equal(ys[r], hys)
        for k in range(eng.nchunks):
            assert bytes(allb[r, k, 21]) == chunk_commits[k]
            for s in range(21):
                assert bytes(allb[r, k, s]) == wits[k * 21 + s], (r, k, s)
    # commit-only pass gives the same chunk commitments
    pts_c, _ = eng.shares(ct, rows, commit_only=True)
    np.testing.assert_array_equal(B.marshal(pts_c).cpu().numpy().reshape(3, eng.nchunks, 64), allb[:, :, 21])
    # compacted full-vector commitment kernel == sum of chunk commitments
    np.testing.assert_array_equal(B.marshal_host(eng.commit_rows(ct, rows)), comm)
    # witness-lanes-only mode (commit_only=2): the same witnesses and share values, slot T not written
    pts_w, ys_w = eng.shares(ct, rows, commit_only=2)
    w_only = B.marshal(pts_w[:, :, :21].contiguous()).cpu().numpy().reshape(3, eng.nchunks, 21, 64)
    np.testing.assert_array_equal(w_only, allb[:, :, :21])
    np.testing.assert_array_equal(ys_w.cpu().numpy(), ys)


def test_sum_rows2_pos_mask_and_early_commitment_sums(rt):
    """bsc_sum_rows2_pos (mask indexed by the position in the row list): the audit's early commitment sums
    over the pre-step's per-peer chunk commitments equal the sums over the share MSM's commitment slots."""
    from biscotti_amd.native import hip
    from biscotti_amd.ops import bn256 as B
    d = 75
    key = rt.CommitKey.generate(d, 3)
    eng = B.DeviceCommitEngine(key, 10, 21)
    rng = np.random.default_rng(5)
    coeffs = torch.from_numpy(rng.integers(-10**4, 10**4, size=(6, d), dtype=np.int64)).cuda()
    ccom, _ = eng.shares(coeffs, torch.arange(6, dtype=torch.int32, device="cuda"), commit_only=True)
    rows = torch.tensor([4, 1, 5, 0], dtype=torch.int32, device="cuda")          # speculative row -> peer row
    mask = torch.tensor([1, 0, 1, 1], dtype=torch.int32, device="cuda")          # alive flags by position
    out = torch.empty((eng.nchunks, 24), dtype=torch.int32, device="cuda")
    assert hip().bsc_sum_rows2_pos(ccom.data_ptr(), eng.nchunks, rows.data_ptr(), 4, None, eng.nchunks,
                                   mask.data_ptr(), out.data_ptr(), None) == 0
    pts, _ = eng.shares(coeffs, rows)                                            # commitment slots = column T
    ref = B.sum_rows(pts.reshape(4, -1, 24), None, torch.arange(eng.nchunks, dtype=torch.int32, device="cuda") * 22 + 21,
                     row_mask=mask)
    np.testing.assert_array_equal(B.marshal(out).cpu().numpy(), B.marshal(ref).cpu().numpy())


@pytest.mark.parametrize("scale,b0", [(3000, 14), (2**40, 14), (2**40, 8), (8193, 14)])
def test_commit_rows_multi_slab(rt, scale, b0):
    """d spanning several 1024-coefficient slabs, zero rows, sparse rows and wide scalars."""
    from biscotti_amd.ops import bn256 as B
    d = 2600
    key = rt.CommitKey.generate(d, 5)
    eng = B.DeviceCommitEngine(key, poly=10, total_shares=21, b0=b0)
    rng = np.random.default_rng(scale % 97)
    coeffs = rng.integers(-scale, scale, size=(4, d), dtype=np.int64)
    coeffs[1] = 0
    coeffs[2, ::7] = 0
    coeffs[3, 1500:] = 0
    rows = torch.tensor([3, 1, 0, 2], dtype=torch.int32, device="cuda")
    got = B.marshal_host(eng.commit_rows(torch.from_numpy(coeffs).cuda(), rows))
    for i, r in enumerate([3, 1, 0, 2]):
        assert bytes(got[i]) == key.commit(coeffs[r], 0), r


def test_sum_rows_is_aggregate(rt):
    from biscotti_amd.ops import bn256 as B
    d = 30
    key = rt.CommitKey.generate(d, 3)
    eng = B.DeviceCommitEngine(key, 10, 21)
    coeffs = np.random.default_rng(1).integers(-10**5, 10**5, size=(4, d), dtype=np.int64)
    pts, _ = eng.shares(torch.from_numpy(coeffs).cuda(), torch.arange(4, dtype=torch.int32, device="cuda"))
    flat = pts.reshape(4, -1, 24)
    rows = torch.tensor([0, 2, 3], dtype=torch.int32, device="cuda")
    agg = B.marshal(B.sum_rows(flat, rows, None)).cpu().numpy().reshape(eng.nchunks, 22, 64)
    summed = coeffs[[0, 2, 3]].sum(0)
    commitment, chunk_commits, hys, wits = key.make_shares(summed, 10, 21)   # homomorphism
    for k in range(eng.nchunks):
        assert bytes(agg[k, 21]) == chunk_commits[k]
        for s in range(21):
            assert bytes(agg[k, s]) == wits[k * 21 + s]


@pytest.mark.parametrize("d,b0", [(57, 11), (7850, 12)])
def test_chunk_check_audits_aggregate(rt, d, b0):
    """k_chunk_check: the recovered aggregate's chunk commitments against the miners' sums of the
    workers' chunk commitments (homomorphism), incl. a short last chunk, wide recovered sums and
    a tampered miner."""
    from biscotti_amd.ops import bn256 as B
    key = rt.CommitKey.generate(d, 3)
    eng = B.DeviceCommitEngine(key, 10, 21, b0=b0)
    rng = np.random.default_rng(d)
    q = rng.integers(-5000, 5000, size=(6, d), dtype=np.int64)
    q[0, :13] = 0
    qt = torch.from_numpy(q).cuda()
    pts, _ = eng.shares(qt, torch.arange(6, dtype=torch.int32, device="cuda"), commit_only=True)   # [6, nch, 1, 24]
    csum = B.sum_rows(pts.reshape(6, eng.nchunks, 24), None, None).view(1, eng.nchunks, 24)
    total = q.sum(0)
    coeffs = np.zeros((eng.nchunks, 10), np.int64)
    coeffs.reshape(-1)[:d] = total
    bad = csum.clone()
    bad[0, 1] = csum[0, 2]                   # miner 1 reports a wrong chunk-1 sum
    both = torch.cat([csum, bad])
    ok = eng.check_chunks(torch.from_numpy(coeffs).cuda(), both).cpu().numpy()
    assert ok[0].all()
    assert ok[1, 1] == 0 and ok[1].sum() == eng.nchunks - 1
    wrong = coeffs.copy()
    wrong[eng.nchunks - 1, 0] += 1
    ok2 = eng.check_chunks(torch.from_numpy(wrong).cuda(), csum).cpu().numpy()
    assert ok2[0, eng.nchunks - 1] == 0 and ok2[0, :-1].all()
    # the device check agrees with the host commitments
    hb = np.stack([np.frombuffer(key.commit(coeffs[k, :min(10, d - 10 * k)], 10 * k), np.uint8)
                   for k in range(eng.nchunks)])
    np.testing.assert_array_equal(B.marshal(csum.view(-1, 24)).cpu().numpy(), hb)


def test_shares_msm_late_cancellation(rt):
    """Rows whose alive flag is cleared are skipped; the others are bit-identical to a full run,
    and set_alive gathers the selection's accept flags onto the speculative rows."""
    from biscotti_amd.ops import bn256 as B
    d = 40
    key = rt.CommitKey.generate(d, 3)
    eng = B.DeviceCommitEngine(key, 10, 21, b0=10)
    q = torch.from_numpy(np.random.default_rng(4).integers(-9000, 9000, size=(4, d), dtype=np.int64)).cuda()
    rows = torch.arange(4, dtype=torch.int32, device="cuda")
    full_p, full_y = eng.shares(q, rows)
    alive = torch.ones(4, dtype=torch.int32, device="cuda")
    # selection rows: accept, reject, accept, accept; speculative rows 0..3 are selection rows 1, none
    # (not a candidate), 0, 3
    B.set_alive(torch.tensor([1, 0, 1, 1], dtype=torch.int32, device="cuda"),
                torch.tensor([1, -1, 0, 3], dtype=torch.int32, device="cuda"), alive)
    assert alive.tolist() == [0, 0, 1, 1]
    p, y = eng.shares(q, rows, alive=alive)
    for r in (2, 3):
        assert torch.equal(p[r], full_p[r]) and torch.equal(y[r], full_y[r])


def test_sum_cols_serial_masked_witness_sums(rt):
    """bsc_sum_cols_serial (the miners' witness sums: one lane per column, kept rows in order) gives the same group
    elements as the LDS-tree form (k_sum_rows2) and as the host's aggregate witnesses (kyber.go:244-287 summed
    homomorphically), with masked rows left out -- including a column set spanning miners' slots and a fully
    masked input (the point at infinity)."""
    from biscotti_amd.native import hip
    from biscotti_amd.ops import bn256 as B
    d = 30
    key = rt.CommitKey.generate(d, 3)
    eng = B.DeviceCommitEngine(key, 10, 21)
    coeffs = np.random.default_rng(2).integers(-10**5, 10**5, size=(5, d), dtype=np.int64)
    pts, _ = eng.shares(torch.from_numpy(coeffs).cuda(), torch.arange(5, dtype=torch.int32, device="cuda"))
    flat = pts.reshape(5, -1, 24).contiguous()
    ncols_in = flat.shape[1]
    cols = torch.tensor([k * 22 + s for k in range(eng.nchunks) for s in (0, 3, 7, 20)], dtype=torch.int32,
                        device="cuda")
    for mask_l in ([1, 0, 1, 1, 0], [0, 0, 0, 0, 0]):
        mask = torch.tensor(mask_l, dtype=torch.int32, device="cuda")
        got = torch.empty((cols.numel(), 24), dtype=torch.int32, device="cuda")
        assert hip().bsc_sum_cols_serial(flat.data_ptr(), ncols_in, 5, cols.data_ptr(), cols.numel(), mask.data_ptr(),
                                         got.data_ptr(), None) == 0
        ref = torch.empty_like(got)
        assert hip().bsc_sum_rows2(flat.data_ptr(), ncols_in, None, 5, cols.data_ptr(), cols.numel(), mask.data_ptr(),
                                   ref.data_ptr(), None) == 0
        np.testing.assert_array_equal(B.marshal(got).cpu().numpy(), B.marshal(ref).cpu().numpy())
        kept = [i for i, m in enumerate(mask_l) if m]
        if kept:
            _, _, _, wits = key.make_shares(coeffs[kept].sum(0), 10, 21)
            g = B.marshal(got).cpu().numpy()
            for i, (k, s) in enumerate((k, s) for k in range(eng.nchunks) for s in (0, 3, 7, 20)):
                assert bytes(g[i]) == wits[k * 21 + s]
        else:
            assert not B.marshal(got).cpu().numpy().any()   # infinity marshals as zeros
