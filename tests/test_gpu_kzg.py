"""Batched verifySecret (K13, kyber.go:650-673) on the device: kzg.hip's random-linear-combination
G1 sums against the host oracle (kzg_rlc_host, same r_kj), and the three-pairing product check over
prepared G2 points accepting honest aggregates and rejecting tampered witnesses / share values."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

T, POLY = 21, 10


def _aggregate(rt, d, secret, contributing, part, spm=7, nrows=4, seed=0):
    """Device shares of random rows summed the way the engine sums them: chunk commitments
    [nch, 24], witnesses [(miner, chunk, slot), 24], share values [nch, npts] at xs."""
    from biscotti_amd.ops import bn256 as B
    key = rt.CommitKey.generate(d, secret)
    eng = B.DeviceCommitEngine(key, POLY, T, b0=10)
    rng = np.random.default_rng(seed)
    coeffs = rng.integers(-10**6, 10**6, size=(nrows, d), dtype=np.int64)
    pts, ys = eng.shares(torch.from_numpy(coeffs).cuda(), torch.arange(nrows, dtype=torch.int32, device="cuda"))
    nch = eng.nchunks
    flat = pts.reshape(nrows, nch * (T + 1), 24)
    base = np.arange(nch) * (T + 1)
    ccols = base + T
    wcols = np.concatenate([(base[:, None] + spm * part[m] + np.arange(spm)[None, :]).reshape(-1) for m in contributing])
    ycols = np.concatenate([spm * part[m] + np.arange(spm) for m in contributing])
    c = lambda a: torch.from_numpy(a.astype(np.int32)).cuda()
    csum = B.sum_rows(flat, None, c(ccols))
    wsum = B.sum_rows(flat, None, c(wcols))
    yagg = ys.sum(0).index_select(1, c(ycols).long()).contiguous()
    xs = c(ycols - 10)
    return key, eng, csum, wsum, yagg, xs, spm


def _host_inputs(rt, key, eng, csum, wsum, yagg, xs, spm, literal):
    nch, npts = yagg.shape
    dev = lambda t: [rt.g1_from_device_jac(r) for r in t.cpu().numpy().view(np.uint32)]
    C = dev(csum)
    Wm = dev(wsum)   # (miner, chunk, slot) order -> (chunk, point) order
    W = [Wm[(j // spm) * nch * spm + k * spm + j % spm] for k in range(nch) for j in range(npts)]
    bases = [rt.g1_generator()] if literal else [key.point(POLY * k) for k in range(nch)]
    return C, W, yagg.cpu().numpy().reshape(-1), xs.cpu().numpy().tolist(), bases


@pytest.mark.parametrize("contributing,part", [([0, 1, 2], {0: 0, 1: 1, 2: 2}), ([2, 0], {2: 0, 0: 2})])
def test_kzg_rlc_matches_host_and_pairing_accepts(rt, contributing, part):
    secret, seed = 2, 0xC0FFEE1234
    key, eng, csum, wsum, yagg, xs, spm = _aggregate(rt, 57, secret, contributing, part)
    out = eng.kzg_rlc(csum, wsum, yagg, xs, spm, literal=False, seed=seed)
    got = [rt.g1_from_device_jac(p) for p in out.cpu().numpy().view(np.uint32)]
    C, W, y, x, bases = _host_inputs(rt, key, eng, csum, wsum, yagg, xs, spm, literal=False)
    assert got == list(rt.kzg_rlc_host(C, W, y, x, bases, seed, 4))
    g2 = rt.g2_generator()
    g2s = rt.g2_mul(g2, secret)
    assert rt.kzg_check(*got, g2, g2s)
    assert rt.kzg_check_device_async(out.cpu().numpy().view(np.uint32), g2, g2s).result()
    # one share checked the reference's way agrees
    assert rt.verify_secret(C[1], W[1 * len(x) + 3], g2, g2s, x[3], int(y[1 * len(x) + 3]), bases[1])


def test_kzg_rejects_tampering(rt):
    secret = 2
    key, eng, csum, wsum, yagg, xs, spm = _aggregate(rt, 57, secret, [0, 1, 2], {0: 0, 1: 1, 2: 2}, seed=1)
    g2 = rt.g2_generator()
    g2s = rt.g2_mul(g2, secret)

    def check(cs, ws, ya, literal=False, seed=99):
        out = eng.kzg_rlc(cs, ws, ya, xs, spm, literal=literal, seed=seed)
        return rt.kzg_check_device_async(out.cpu().numpy().view(np.uint32), g2, g2s).result()

    assert check(csum, wsum, yagg)
    w2 = wsum.clone()
    w2[5] = wsum[6]                      # one witness swapped for its neighbour's
    assert not check(csum, w2, yagg)
    y2 = yagg.clone()
    y2[3, 4] += 1                        # one share value off by one
    assert not check(csum, wsum, y2)
    c2 = csum.clone()
    c2[2] = csum[1]                      # one chunk commitment replaced
    assert not check(c2, wsum, yagg)
    # the literal check (y against G1) only holds for chunk 0 (quirk Q9)
    assert not check(csum, wsum, yagg, literal=True)


def test_kzg_literal_single_chunk(rt):
    key, eng, csum, wsum, yagg, xs, spm = _aggregate(rt, 10, 2, [0, 1, 2], {0: 1, 1: 2, 2: 0}, seed=2)
    assert eng.nchunks == 1
    out = eng.kzg_rlc(csum, wsum, yagg, xs, spm, literal=True, seed=5)
    g2 = rt.g2_generator()
    assert rt.kzg_check_device_async(out.cpu().numpy().view(np.uint32), g2, rt.g2_mul(g2, 2)).result()


@pytest.mark.parametrize("mode", ["consistent", "literal"])
def test_engine_kzg_audit_on_gpu(mode):
    """The engine's per-round KZG audit on the device path (MNIST, 785 chunks x 21 points per round):
    consistent passes every block, literal fails every block (quirk Q9); the chain is unaffected."""
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    cfg = RunConfig(num_nodes=20, seed=3, deterministic_time=True, kzg_audit=mode, max_iterations=100)
    eng = BiscottiEngine(cfg, Comm(device=torch.device("cuda", 0)))
    try:
        res = [eng.run_round() for _ in range(6)]
        eng.drain()
        blocks = sum(1 for r in res if r is not None and not r.empty)
        assert blocks >= 4
        assert eng.stats["kzg_checks"] == blocks
        assert eng.stats["kzg_failures"] == (0 if mode == "consistent" else blocks)
        assert eng.fsm.chain.verify()[0]
    finally:
        eng.close()
