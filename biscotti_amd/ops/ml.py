"""Learning-side ops of a Biscotti round: local step, DP noise, Multi-Krum, evaluation, recovery.

On a GPU every op launches the gfx950 kernel from ``csrc/kernels/ml.hip`` (there is no eager
fallback on GPU: a missing library raises).  On CPU the same math runs as a numpy/torch reference
that draws from the identical Philox4x32-10 streams, so CPU runs reproduce GPU runs up to
float rounding and GPU numerics tests compare against it.
"""
from __future__ import annotations

import numpy as np
import torch

from ..native import hip
from ..utils import pinned
from ..utils import streams as S

PHILOX_M0, PHILOX_M1 = 0xD2511F53, 0xCD9E8D57
PHILOX_W0, PHILOX_W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = 0xFFFFFFFF


def _stream() -> int:
    return S.raw()


def _p(t):
    if t is None:
        return None
    assert t.is_contiguous(), "kernel operands must be contiguous"
    return t.data_ptr()


def _check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"HIP launch of {what} failed (code {err})")


# ---------------------------------------------------------------------------- Philox (numpy)
def philox4x32(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10; inputs are uint32-compatible arrays/scalars."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint64) & MASK32 for v in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (x.copy() for x in (c0, c1, c2, c3))
    k0 = np.uint64(k0 & MASK32)
    k1 = np.uint64(k1 & MASK32)
    for _ in range(10):
        p0 = np.uint64(PHILOX_M0) * c0
        p1 = np.uint64(PHILOX_M1) * c2
        n0 = ((p1 >> np.uint64(32)) ^ c1 ^ k0) & np.uint64(MASK32)
        n1 = p1 & np.uint64(MASK32)
        n2 = ((p0 >> np.uint64(32)) ^ c3 ^ k1) & np.uint64(MASK32)
        n3 = p0 & np.uint64(MASK32)
        c0, c1, c2, c3 = n0, n1, n2, n3
        k0 = np.uint64((int(k0) + PHILOX_W0) & MASK32)
        k1 = np.uint64((int(k1) + PHILOX_W1) & MASK32)
    return c0, c1, c2, c3


def _u01(v):
    return ((np.asarray(v) >> np.uint64(8)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)


def _gauss(a, b):
    r = np.sqrt(np.float32(-2.0) * np.log(_u01(a)))
    return (r * np.cos(np.float32(6.28318530717958647692) * _u01(b))).astype(np.float32)


def minibatch_indices(p: int, iteration: int, n: int, B: int, seed: int, tag: int = 0x5EED) -> list[int]:
    """The B distinct indices the local-step kernel draws for peer p (DataLoader shuffle analogue)."""
    out: list[int] = []
    ctr = 0
    while len(out) < min(B, n):
        r = philox4x32(p, iteration, ctr, tag, seed & MASK32, (seed >> 32) & MASK32)
        ctr += 1
        for v in r:
            if len(out) >= min(B, n):
                break
            c = int(v) % n
            if c not in out:
                out.append(c)
    return out


# ---------------------------------------------------------------------------- K1 softmax step
def softmax_step(X, y, off, ntrain, pid, W, d_in, d_out, B, seed, iteration, max_norm=100.0, qscale=1e4, lo=-1):
    """Batched local SGD step of SoftmaxModel for every local peer.

    X fp32 [Ntot, d_in]; y int32 [Ntot]; off int64 [P]; ntrain int32 [P]; pid int32 [P] global peer
    ids (key of each peer's minibatch stream); W fp64 [nparam].  lo >= 0: off / ntrain are indexed by
    local peer id pid - lo (resident arrays over all local peers) instead of by row.
    Returns (delta fp32 [P, nparam] = -clip(grad), qdelta int64 [P, nparam], loss fp32 [P]).
    """
    P = pid.numel()
    nparam = d_out * d_in + d_out
    dev = X.device
    delta = torch.empty((P, nparam), dtype=torch.float32, device=dev)
    qdelta = torch.empty((P, nparam), dtype=torch.int64, device=dev)
    loss = torch.empty((P,), dtype=torch.float32, device=dev)
    if dev.type == "cuda":
        assert X.dtype == torch.float32 and y.dtype == torch.int32 and W.dtype == torch.float64
        assert off.dtype == torch.int64 and ntrain.dtype == torch.int32 and W.numel() == nparam
        assert pid.dtype == torch.int32 and (lo >= 0 or off.numel() == P)
        _check(hip().bsc_softmax_step(_p(X), _p(y), _p(off), _p(ntrain), _p(pid), _p(W), d_in, d_out, B, P, seed & (2**64 - 1),
                                      iteration, float(max_norm), float(qscale), _p(delta), _p(qdelta), _p(loss),
                                      int(lo), _stream()), "softmax_step")
        return delta, qdelta, loss
    Wm = W.to(torch.float32)
    Wt, bt = Wm[: d_out * d_in].view(d_out, d_in), Wm[d_out * d_in:]
    pids = pid.tolist()
    if lo >= 0:
        offs = [int(off[q - lo]) for q in pids]
        ns = [int(ntrain[q - lo]) for q in pids]
    else:
        offs, ns = off.tolist(), ntrain.tolist()
    for p in range(P):
        idx = minibatch_indices(pids[p], iteration, ns[p], B, seed)
        rows = torch.tensor([offs[p] + i for i in idx], dtype=torch.long)
        xb = (X[rows] - 0.5) / 0.5
        logits = xb @ Wt.T + bt
        lab = y[rows].long()
        lossv = torch.nn.functional.cross_entropy(logits, lab)
        g = (torch.softmax(logits, 1) - torch.nn.functional.one_hot(lab, d_out).float()) / len(idx)
        dW, db = g.T @ xb, g.sum(0)
        flat = torch.cat([dW.reshape(-1), db])
        tot = float(torch.linalg.vector_norm(flat))
        coef = max_norm / (tot + 1e-6)
        if coef < 1:
            flat = flat * coef
        v = -flat
        delta[p] = v
        qdelta[p] = torch.from_numpy((v.double().numpy() * qscale).astype(np.int64))
        loss[p] = lossv
    return delta, qdelta, loss


# ---------------------------------------------------------------------------- K3 logistic step
def logreg_step(X, y, off, nrows, pid, W, B, seed, calls, alpha, lammy, sigma, qscale=1e4):
    """Batched logistic-regression step (creditcard path), DP noise at source when sigma > 0.

    X fp64 [Ntot, D]; y fp64 [Ntot] (+-1); off int64 [P]; nrows int32 [P]; W fp64 [D];
    calls int32 [P] (per-peer privateFun call counter); sigma fp64 [P].
    """
    P, D = off.numel(), X.shape[1]
    dev = X.device
    delta = torch.empty((P, D), dtype=torch.float32, device=dev)
    qdelta = torch.empty((P, D), dtype=torch.int64, device=dev)
    if dev.type == "cuda":
        _check(hip().bsc_logreg_step(_p(X), _p(y), _p(off), _p(nrows), _p(pid), _p(W), D, B, P, seed & (2**64 - 1), _p(calls),
                                     float(alpha), float(lammy), _p(sigma), float(qscale), _p(delta), _p(qdelta),
                                     _stream()), "logreg_step")
        return delta, qdelta
    Xn, yn, Wn = X.numpy(), y.numpy(), W.numpy()
    for p in range(P):
        n = int(nrows[p])
        idx = minibatch_indices(int(pid[p]), int(calls[p]), n, B, seed, tag=0x106)
        rows = [int(off[p]) + i for i in idx]
        xb, yb = Xn[rows], yn[rows]
        t = yb * (xb @ Wn)
        res = -yb / np.exp(np.logaddexp(0, t))
        g = xb.T @ res / B + lammy * Wn
        v = -alpha * g
        if float(sigma[p]) > 0:
            r = philox4x32(np.arange(D), int(calls[p]) % 100, int(pid[p]), 0xD9, (seed >> 7) & MASK32, (seed >> 39) & MASK32)
            v = v + (-alpha / B) * float(sigma[p]) * np.sqrt(B) * _gauss(r[0], r[1]).astype(np.float64)
        delta[p] = torch.from_numpy(v.astype(np.float32))
        qdelta[p] = torch.from_numpy((v * qscale).astype(np.int64))
    return delta, qdelta


# ---------------------------------------------------------------------------- K4 DP noise
def noise_table(num_noisers: int, D: int, seed: int, device) -> torch.Tensor:
    """Every noiser's 100 pre-sampled N(0,1) vectors, resident on the device: fp32
    [num_noisers, 100, D] (client_obj.py:61-63 pre-samples samples[100][D] per peer at init).
    Entry [j, m] equals the vector dp_noise draws for noiser j at iterations = m (mod 100)."""
    tbl = torch.empty((num_noisers, 100, D), dtype=torch.float32, device=device)
    _check(hip().bsc_noise_table(num_noisers, D, seed & (2**64 - 1), _p(tbl), _stream()), "noise_table")
    return tbl


def dp_noise(delta, noisers, scales, seed, iteration, table=None, rows=None):
    """noised = delta + mean_j scales[p, j] * N(0, 1; noiser_j, iteration % 100).

    `table` (GPU): the resident noise_table of the same seed -- the kernel then gathers the
    noisers' vectors instead of regenerating them (identical values).  `rows` (int32, GPU, needs
    `table`): return only those rows, in that order (fused gather); the caller validated them."""
    P, D = delta.shape
    nn_ = noisers.shape[1] if noisers.dim() == 2 else 0
    if delta.device.type == "cuda":
        if table is not None:
            assert table.shape[1:] == (100, D) and table.dtype == torch.float32
            if nn_ and P and noisers.device.type == "cpu":
                assert int(noisers.min()) >= 0 and int(noisers.max()) < table.shape[0], "noiser id out of range"
            # device-resident ids: the caller range-checks them on the host (reading them back here
            # would stall the stream)
            assert rows is None or rows.dtype == torch.int32
            n_out = P if rows is None else rows.numel()
            out = torch.empty((n_out, D), dtype=delta.dtype, device=delta.device)
            _check(hip().bsc_dp_noise_tbl(_p(delta), n_out, D, _p(noisers), nn_, _p(scales), _p(table),
                                          iteration % 100, _p(rows), _p(out), _stream()), "dp_noise_tbl")
            return out
        out = torch.empty_like(delta)
        _check(hip().bsc_dp_noise(_p(delta), P, D, _p(noisers), nn_, _p(scales), seed & (2**64 - 1), iteration % 100,
                                  _p(out), _stream()), "dp_noise")
        return out
    acc = np.zeros((P, D), dtype=np.float32)
    idx = np.arange(D)
    for p in range(P):
        for j in range(nn_):
            nid = int(noisers[p, j])
            r = philox4x32(idx, iteration % 100, nid, 0xA11CE, seed & MASK32, (seed >> 32) & MASK32)
            acc[p] += np.float32(float(scales[p, j])) * _gauss(r[0], r[1])
    if nn_:
        acc /= np.float32(nn_)
    return delta + torch.from_numpy(acc)


def noise_vector(noiser: int, iteration: int, D: int, seed: int) -> np.ndarray:
    """N(0,1) vector a noiser contributes at `iteration` (before scaling) -- RequestNoise payload."""
    r = philox4x32(np.arange(D), iteration % 100, noiser, 0xA11CE, seed & MASK32, (seed >> 32) & MASK32)
    return _gauss(r[0], r[1])


class NoiseRows:
    """Every noiser's 100 pre-sampled N(0,1) vectors (client_obj.py:61-63 pre-samples samples[100][D] per
    peer at init): rows(it) -> fp32 [N, D] whose row j is the vector noiser j contributes at iteration
    it (mod 100), before scaling.  GPU: ONE resident table [N, 100, D] (noise_table; 314 MB for MNIST x
    100 peers), rows() a strided view.  CPU: generated per iteration from the same Philox stream
    (bit-identical to dp_noise's regeneration) and cached for the last iteration."""

    def __init__(self, N: int, D: int, seed: int, device):
        self.N, self.D, self.seed = N, D, seed
        self.device = torch.device(device)
        self.table = noise_table(N, D, seed, device) if self.device.type == "cuda" else None
        self._m, self._rows = None, None

    def rows(self, it: int) -> torch.Tensor:
        m = it % 100
        if self.table is not None:
            return self.table[:, m, :]
        if self._m != m:
            r = philox4x32(np.arange(self.D)[None, :], m, np.arange(self.N)[:, None], 0xA11CE, self.seed & MASK32,
                           (self.seed >> 32) & MASK32)
            self._rows, self._m = torch.from_numpy(_gauss(r[0], r[1])), m
        return self._rows

    def gram_table(self, kchunk: int = 512) -> torch.Tensor:
        """GPU: [100, N, N] fp64, entry [m, a, b] = <rows(m)[a], rows(m)[b]> as k_gram_pairs computes it (the same
        kernel, K split and reduction order, so the noise-aware Gram's noise x noise tiles copied from here are
        bit-identical to computed ones).  The noisers' vectors repeat with the iteration mod 100
        (client_obj.py:61-63,97-98): built once (~8 MB at N = 100), a setup cost instead of ~23 % of every
        round's Gram tiles."""
        tab = getattr(self, "_gram_tab", None)
        if tab is not None:
            return tab
        assert self.table is not None, "the noise Gram table lives on the GPU"
        N, D, dev = self.N, self.D, self.device
        T = (N + 15) // 16
        npairs, nsplit = T * (T + 1) // 2, (D + kchunk - 1) // kchunk
        part = torch.empty((nsplit, npairs, 256), dtype=torch.float64, device=dev)
        tiles = torch.empty((npairs, 256), dtype=torch.float64, device=dev)
        cnt = _tile_counters(dev, npairs)
        # (pair, e) -> (a, b) of the dense matrix, both triangles
        pr = torch.tensor(_pair_tiles(T), dtype=torch.long)
        e = torch.arange(256)
        a = (pr[:, 0, None] * 16 + e[None, :] // 16).reshape(-1)
        b = (pr[:, 1, None] * 16 + e[None, :] % 16).reshape(-1)
        ok = (a < N) & (b < N)
        src = torch.nonzero(ok).flatten().to(dev)
        ia, ib = a[ok].to(dev), b[ok].to(dev)
        tab = torch.empty((100, N, N), dtype=torch.float64, device=dev)
        for m in range(100):
            rows = self.table[:, m, :]
            _check(hip().bsc_gram_stacked_range(None, 0, rows.data_ptr(), N, rows.stride(0), D, kchunk, 0, 0,
                                                _p(part), _p(tiles), _p(cnt), None, _stream()), "gram_noise_table")
            flat = tiles.view(-1).index_select(0, src)
            tab[m].index_put_((ia, ib), flat)
            tab[m].index_put_((ib, ia), flat)
        self._gram_tab = tab
        return tab


# ---------------------------------------------------------------------------- K5 Multi-Krum
def krum_async(X, groupsize: int, n_accept: int, ksplit: int = 256, on_accept=None):
    """Queue Multi-Krum over the rows of X (fp32 [n, d], GPU); returns a callable giving
    (accept bool [n] on the host, scores fp64 [n] on the device).

    The selection is downloaded right behind its kernel, so the callable waits for Krum only --
    not for work queued later on the stream.  on_accept(acc_int32) is called right after the
    selection kernel is queued (e.g. to cancel or aggregate speculative work on the device)."""
    n, D = X.shape
    assert X.device.type == "cuda" and 0 < n <= 128, "krum kernel handles 1..128 updates per verifier"
    tiles = (n + 15) // 16
    nsplit = (D + ksplit - 1) // ksplit
    part = torch.empty((nsplit, tiles * 16, tiles * 16), dtype=torch.float64, device=X.device)
    dist = torch.empty((n, n), dtype=torch.float64, device=X.device)
    scores = torch.empty((n,), dtype=torch.float64, device=X.device)
    acc = torch.empty((n,), dtype=torch.int32, device=X.device)
    _check(hip().bsc_krum(_p(X), n, D, ksplit, _p(part), _p(dist), _p(scores), _p(acc), groupsize, n_accept,
                          _stream()), "krum")
    host = torch.empty(acc.shape, dtype=acc.dtype, pin_memory=True)
    host.copy_(acc, non_blocking=True)
    ev = S.record()
    if on_accept is not None:
        on_accept(acc)

    def result():
        S.host_wait(ev)
        return host.bool(), scores
    return result


def krum(X, groupsize: int, n_accept: int, ksplit: int = 256, on_accept=None):
    """Multi-Krum over the rows of X (fp32 [n, d]): returns (accept bool [n], scores fp64 [n]).

    on_accept(acc_int32) (GPU): see krum_async."""
    n, D = X.shape
    if n == 0:
        return torch.zeros(0, dtype=torch.bool), torch.zeros(0, dtype=torch.float64)
    if X.device.type == "cuda":
        return krum_async(X, groupsize, n_accept, ksplit, on_accept)()
    Xd = X.double()
    sq = (Xd * Xd).sum(1)
    dist = sq[:, None] + sq[None] - 2 * Xd @ Xd.T
    srt, _ = torch.sort(dist, dim=1)
    hi = max(1, min(groupsize - 1, n))
    scores = srt[:, 1:hi].sum(1) if hi > 1 else torch.zeros(n, dtype=torch.float64)
    order = sorted(range(n), key=lambda i: (float(scores[i]), i))
    acc = torch.zeros(n, dtype=torch.bool)
    acc[order[:n_accept]] = True
    return acc, scores


def _gram_exact_order(S: torch.Tensor) -> torch.Tensor:
    """fp64 Gram of the rows of S with every entry reduced in ONE fixed order whatever the number of rows:
    exact products (fp32 x fp32 fits fp64), then a pairwise tree of element-wise adds over the
    zero-padded inner dimension.  A candidate pair therefore gets bit-identical distances on one rank
    and on several (different row sets), which a BLAS GEMM -- blocked by matrix size and threads --
    does not guarantee."""
    S = S.double().cpu()
    U, D = S.shape
    Dp = 1 << max(0, (max(D, 1) - 1).bit_length())
    Sp = torch.zeros((U, Dp), dtype=torch.float64)
    Sp[:, :D] = S
    G = torch.empty((U, U), dtype=torch.float64)
    for i in range(U):
        P = Sp[i][None, :] * Sp
        while P.shape[1] > 1:
            h = P.shape[1] // 2
            P = P[:, :h] + P[:, h:]
        G[i] = P[:, 0]
    return G


def _committee_host(X, inbox, groupsize, n_accept, need, lead_rank, cap, G=None):
    """fp64 torch reference of the committee Krum (same tie-breaks as the kernels).  G: the candidates'
    fp64 Gram when the caller has it (the noise-aware form assembles it), else X X^T."""
    ib = inbox.cpu().long()
    V, n = ib.shape
    if G is None:
        G = _gram_exact_order(X)
    U = G.shape[0]
    sq = torch.diagonal(G)
    acc = torch.zeros((V, n), dtype=torch.bool)
    sigs = torch.zeros((U,), dtype=torch.long)
    hi = max(1, min(groupsize - 1, n))
    for v in range(V):
        rows = ib[v]
        D = sq[rows][:, None] + sq[rows][None] - 2 * G[rows][:, rows]
        srt, _ = torch.sort(D, dim=1)
        sc = srt[:, 1:hi].sum(1) if hi > 1 else torch.zeros(n, dtype=torch.float64)
        order = sorted(range(n), key=lambda i: (float(sc[i]), i))
        acc[v, order[:n_accept]] = True
        sigs.index_add_(0, rows[acc[v]], torch.ones(int(acc[v].sum()), dtype=torch.long))
    lr = lead_rank.cpu().long()
    appr = (lr >= 0) & (sigs >= need)
    node = appr.clone()
    if cap > 0 and int(appr.sum()) > cap:
        idx = [int(w) for w in torch.nonzero(appr).flatten()]
        idx.sort(key=lambda w: int(lr[w]))
        node[:] = False
        node[idx[:cap]] = True
    return acc, node


KRUM_MAX_ROWS = 8192    # committee Krum: candidate rows (Gram operand rows)
KRUM_MAX_INBOX = 4096   # committee Krum: updates per verifier inbox

_COUNTERS: dict = {}


def _tile_counters(dev, n: int) -> torch.Tensor:
    """Zeroed per-tile arrival counters of the in-kernel split-K reduction; the kernel re-arms them,
    so one buffer per device serves every launch (stream-ordered on the round's main stream)."""
    key = (str(dev), S.raw())
    buf = _COUNTERS.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.zeros((max(n, 1024),), dtype=torch.int32, device=dev)
        _COUNTERS[key] = buf
    return buf


def krum_committee_async(X, inbox, groupsize: int, n_accept: int, need: int, lead_rank, cap: int,
                         kchunk: int = 512, on_accept=None):
    """Multi-Krum of a whole verifier committee in one pass (the reference runs Krum once per
    verifier process on that verifier's own inbox, krum.go:284-322).

    X fp32 [U, d]: the candidate rows (submitted workers' noised deltas); inbox int32 [V, n]: each
    live verifier's inbox as rows of X (sorted by SourceID); lead_rank int32 [U]: arrival rank of
    each row at the leader miner (-1: row is not a submitted worker); need = floor(nv / 2)
    signatures; cap = NUM_SAMPLES/2 leader threshold (0: no cap).

    Returns a callable giving (acc bool [V, n], node bool [U]) on the host: acc[v, i] = verifier v
    signs inbox[v, i]; node = rows the leader's block carries.  On a GPU on_accept(node_int32) is
    called with the device mask right after the vote kernel is queued."""
    U, D = X.shape
    V, n = inbox.shape
    if X.device.type != "cuda":
        acc, node = _committee_host(X, inbox, groupsize, n_accept, need, lead_rank, cap)
        if on_accept is not None:
            on_accept(node.to(torch.int32))
        return lambda: (acc, node)
    assert X.dtype == torch.float32 and inbox.dtype == torch.int32 and lead_rank.dtype == torch.int32
    assert 0 < U <= KRUM_MAX_ROWS and 0 < n <= KRUM_MAX_INBOX and 0 < V <= 64 and n <= U, "committee Krum size limits"
    assert lead_rank.numel() == U
    T = (U + 15) // 16
    npairs = T * (T + 1) // 2
    nsplit = (D + kchunk - 1) // kchunk
    dev = X.device
    part = torch.empty((nsplit, npairs, 256), dtype=torch.float64, device=dev)
    gram = torch.empty((npairs, 256), dtype=torch.float64, device=dev)
    count = _tile_counters(dev, npairs)
    scores = torch.empty((V, n), dtype=torch.float64, device=dev)
    out = torch.empty((V * n + U,), dtype=torch.int32, device=dev)
    acc, node = out[: V * n], out[V * n:]
    ws = torch.empty((U,), dtype=torch.int32, device=dev) if (U > 1024 or n > 256) else None
    _check(hip().bsc_krum_committee(_p(X.contiguous()), U, D, kchunk, _p(inbox.contiguous()), V, n, groupsize, n_accept,
                                    need, _p(lead_rank.contiguous()), cap, _p(part), _p(gram), _p(count), _p(scores),
                                    _p(acc), _p(node), _p(ws), _stream()), "krum_committee")
    host = torch.empty(out.shape, dtype=torch.int32, pin_memory=True)
    host.copy_(out, non_blocking=True)
    ev = S.record()
    if on_accept is not None:
        on_accept(node)

    def result():
        S.host_wait(ev)
        h = host.bool()
        return h[: V * n].view(V, n), h[V * n:]
    return result


def _pair_tiles(T: int) -> list[tuple[int, int]]:
    """(ti, tj) of every tile pair ti <= tj of a T x T tile grid, in k_gram_pairs' enumeration order."""
    return [(ti, tj) for ti in range(T) for tj in range(ti, T)]


def _gram_tiles_exact(S: torch.Tensor, p0: int, p1: int, T: int) -> torch.Tensor:
    """CPU: tiles [p0, p1) of the tiled upper-triangular Gram ([p1 - p0, 256] fp64, entry [p, 16 a + b] =
    G[16 ti + a, 16 tj + b]) with every entry reduced exactly as _gram_exact_order reduces it."""
    S = S.double().cpu()
    U, D = S.shape
    Dp = 1 << max(0, (max(D, 1) - 1).bit_length())
    Sp = torch.zeros((T * 16, Dp), dtype=torch.float64)
    Sp[:U, :D] = S
    out = torch.zeros((p1 - p0, 256), dtype=torch.float64)
    for k, (ti, tj) in enumerate(_pair_tiles(T)[p0:p1]):
        B_ = Sp[tj * 16:(tj + 1) * 16]
        for a in range(16):
            P = Sp[ti * 16 + a][None, :] * B_
            while P.shape[1] > 1:
                h = P.shape[1] // 2
                P = P[:, :h] + P[:, h:]
            out[k, a * 16:(a + 1) * 16] = P[:, 0]
    return out


def gram_full_from_tiles(tiles: torch.Tensor, U: int) -> torch.Tensor:
    """The symmetric [U, U] Gram out of its tiled upper triangle ([npairs, 256], k_gram_pairs' layout)."""
    T = (U + 15) // 16
    G = torch.zeros((T * 16, T * 16), dtype=torch.float64)
    for k, (ti, tj) in enumerate(_pair_tiles(T)):
        t = tiles[k].double().cpu().view(16, 16)
        G[ti * 16:(ti + 1) * 16, tj * 16:(tj + 1) * 16] = t
        G[tj * 16:(tj + 1) * 16, ti * 16:(ti + 1) * 16] = t.T
    return G[:U, :U].contiguous()


def gram_split(U: int, rank: int, world: int) -> tuple[int, int, int, int]:
    """(p0, p1, chunk, npairs): the tile pairs [p0, p1) of a U-row Gram that `rank` of `world` computes.
    Rank r owns [r * chunk, (r + 1) * chunk) clipped to npairs, so the ranks' [chunk, 256] slots
    all_gathered in rank order start with the whole tiled Gram."""
    T = (U + 15) // 16
    npairs = T * (T + 1) // 2
    chunk = -(-npairs // world)
    p0 = min(npairs, rank * chunk)
    return p0, min(npairs, p0 + chunk), chunk, npairs


def gram_stacked_async(X, T_rows, kchunk: int = 512, split: tuple[int, int] | None = None, out=None,
                       nn=None) -> dict:
    """Noise-aware committee Krum, phase 1: f64 Gram of the stacked rows [X; T_rows].

    X fp32 [U1, d] (the workers' deltas, contiguous); T_rows fp32 [U2, d] with contiguous rows (a
    strided view of the resident noise table at this iteration).  Runs before the noisers are known.
    split = (rank, world): this rank computes only its share of the tile pairs (gram_split) into rows
    [rank * chunk, ...) of a [world * chunk, 256] buffer; the caller all_gathers the ranks' slots
    (gram_slot) and calls gram_adopt.  out (GPU, split): this rank's [chunk, 256] slot is written there
    instead (the packed verification row, ops/gather.py).  nn (GPU): this iteration's dense [U2, U2] Gram of
    T_rows (NoiseRows.gram_table): the noise x noise tiles are copied from it, not computed.  Returns the
    handle krum_committee_noise_async consumes."""
    U1, D = X.shape
    U2 = T_rows.shape[0]
    assert X.is_contiguous() and T_rows.stride(1) == 1 and T_rows.shape[1] == D
    assert X.dtype == torch.float32 and T_rows.dtype == torch.float32
    U = U1 + U2
    assert 0 < U <= KRUM_MAX_ROWS, "committee Krum size limits"
    Tt = (U + 15) // 16
    npairs = Tt * (Tt + 1) // 2
    if split is not None:
        rank, world = split
        p0, p1, chunk, _ = gram_split(U, rank, world)
    else:
        rank, p0, p1, chunk = 0, 0, npairs, npairs
    if X.device.type != "cuda":
        if split is None:
            return {"gram_full": _gram_exact_order(torch.cat([X, T_rows])), "U1": U1, "U": U}
        slots = torch.zeros((chunk * split[1], 256), dtype=torch.float64)
        slots[rank * chunk:rank * chunk + (p1 - p0)] = _gram_tiles_exact(torch.cat([X, T_rows]), p0, p1, Tt)
        return {"gram": slots, "U1": U1, "U": U, "split": (rank, chunk, npairs)}
    nsplit = (D + kchunk - 1) // kchunk
    dev = X.device
    part = torch.empty((nsplit, max(1, p1 - p0), 256), dtype=torch.float64, device=dev)
    if out is not None:
        assert split is not None and out.dtype == torch.float64 and tuple(out.shape) == (chunk, 256)
        gram = out
        base = out.data_ptr() - p0 * 256 * 8   # the kernel indexes its output by the global pair index
    else:
        gram = torch.empty((chunk * (split[1] if split else 1), 256), dtype=torch.float64, device=dev)
        base = gram.data_ptr()
    _check(hip().bsc_gram_stacked_range(_p(X), U1, T_rows.data_ptr(), U2, T_rows.stride(0), D, kchunk, p0, p1,
                                        _p(part), base, _p(_tile_counters(dev, max(1, p1 - p0))),
                                        nn.data_ptr() if nn is not None else None, _stream()),
           "gram_stacked")
    res = {"gram": gram, "U1": U1, "U": U, "keep": (X, T_rows, part)}
    if split is not None:
        res["split"] = (rank, chunk, npairs)
        if out is not None:
            res["packed"] = True
    return res


def gram_slot(pre: dict) -> torch.Tensor:
    """This rank's [chunk, 256] slot of a split Gram (the part it sends)."""
    rank, chunk, _ = pre["split"]
    return pre["gram"][rank * chunk:(rank + 1) * chunk]


def gram_adopt(pre: dict, gathered: torch.Tensor) -> None:
    """Install the all_gathered slots [world, chunk, 256] of a split Gram as the whole Gram."""
    _, chunk, npairs = pre["split"]
    full = gathered.reshape(-1, 256)[:npairs]
    if full.device.type != "cuda":
        pre["gram_full"] = gram_full_from_tiles(full, pre["U"])
    pre["gram"] = full
    del pre["split"]


NOISE_ARG_MAX = 400   # kernels/ml.hip: noiser table entries the Krum rows kernel takes in its argument block


def noise_tables_by_value(entries: int, n: int) -> bool:
    """The noisers' ids / weights (entries = U1 * nn) fit the rows kernel's argument block (inbox n <= 256)."""
    return 0 < entries <= NOISE_ARG_MAX and 0 < n <= 256


_KRUM_BUF: dict = {}   # (V, n, U1, device) -> resident outputs of krum_committee_noise_async


def krum_committee_noise_async(pre: dict, nz, sc, inbox, groupsize: int, n_accept: int, need: int, lead_rank,
                               cap: int, on_accept=None, flags=None):
    """Noise-aware committee Krum, phase 2: the noised rows x_a = delta_a + mean_s sc[a, s] t_{nz[a, s]}
    are never materialised -- their inner products are assembled from the phase-1 Gram.  nz int32 /
    sc fp32 [U1, nn] (nz indexes the stacked noise rows) -- device tensors, or (GPU, noise_tables_by_value)
    host numpy arrays that travel in the rows kernel's arguments; the rest as krum_committee_async.  The vote
    kernel writes its verdicts straight into the pinned read-back buffer; flags = (amap, alive): it also sets
    the speculative share MSM's row flags from the block mask (alive[i] = node[amap[i]])."""
    U1, U = pre["U1"], pre["U"]
    V, n = inbox.shape
    nn = nz.shape[1]
    host_tabs = isinstance(nz, np.ndarray)
    if host_tabs:
        nz = np.ascontiguousarray(nz, np.int32)
        sc = np.ascontiguousarray(sc, np.float32)
        assert "gram_full" not in pre and tuple(nz.shape) == (U1, nn) and noise_tables_by_value(nz.size, n)
    assert inbox.dtype == torch.int32 and lead_rank.dtype == torch.int32 and lead_rank.numel() == U1
    assert host_tabs or (nz.dtype == torch.int32 and sc.dtype == torch.float32 and tuple(nz.shape) == (U1, nn))
    assert 0 < n <= KRUM_MAX_INBOX and 0 < V <= 64 and n <= U1 and 0 < nn <= 16
    if "gram_full" in pre:   # CPU: the same assembly as k_krum_rows_noise, term by term in its order
        G, inv = pre["gram_full"], 1.0 / nn
        z, w = nz.long(), sc.double()
        Gx = G[:U1, :U1].clone()
        for t in range(nn):
            Gx += inv * w[None, :, t] * G[:U1, U1 + z[:, t]]
            Gx += inv * w[:, None, t] * G[U1 + z[:, t], :U1]
        for s_ in range(nn):
            for t in range(nn):
                Gx += inv * inv * w[:, None, s_] * w[None, :, t] * G[(U1 + z[:, s_])[:, None], (U1 + z[:, t])[None, :]]
        acc, node = _committee_host(None, inbox, groupsize, n_accept, need, lead_rank, cap, G=Gx)
        if on_accept is not None:
            on_accept(node.to(torch.int32))
        return lambda: (acc, node)
    dev = pre["gram"].device
    # resident outputs per shape (the launches are ordered on the caller's stream; the round reads the verdicts
    # from the pinned copy): no allocator calls on the round's path
    key = (V, n, U1, str(dev))
    buf = _KRUM_BUF.get(key)
    if buf is None:
        out_ = torch.empty((V * n + U1,), dtype=torch.int32, device=dev)
        buf = _KRUM_BUF[key] = (torch.empty((V, n), dtype=torch.float64, device=dev), out_, out_[: V * n],
                                out_[V * n:], torch.empty((U1,), dtype=torch.int32, device=dev)
                                if (U1 > 1024 or n > 256) else None)
    scores, out, acc, node, ws = buf
    host = pinned("krum_noise", out.shape, torch.int32)   # rotating: the last verdicts may still be read
    amap, alive = flags if flags is not None else (None, None)
    fn = hip().bsc_krum_committee_noise_ka if host_tabs else hip().bsc_krum_committee_noise2
    _check(fn(_p(pre["gram"]), U1, U, nz.ctypes.data if host_tabs else _p(nz.contiguous()),
              sc.ctypes.data if host_tabs else _p(sc.contiguous()), nn, _p(inbox.contiguous()), V, n, groupsize,
              n_accept, need, _p(lead_rank.contiguous()), cap, _p(scores), _p(acc), _p(node), _p(ws),
              host.data_ptr(), _p(amap), alive.numel() if alive is not None else 0, _p(alive), _stream()),
           "krum_committee_noise")
    ev = S.record()
    if on_accept is not None:
        on_accept(node)

    def result():
        S.host_wait(ev)
        h = host.bool()
        return h[: V * n].view(V, n), h[V * n:]
    return result


# ---------------------------------------------------------------------------- K2 evaluation
_EVAL_DEV: dict = {}   # pinned read-back buffer -> its device accumulator (persistent pairs)


def eval_tiles(X: torch.Tensor, transform: bool = True) -> torch.Tensor:
    """The test set in k_eval_error_t's layout: [ceil(N/16), ceil(d_in/4), 64] fp32, entry [t, g, l] =
    transform(X[16 t + (l & 15), 4 g + (l >> 4)]) with zero padding (built once per task)."""
    N, D = X.shape
    T, KG = (N + 15) // 16, (D + 3) // 4
    Xp = torch.zeros((T * 16, KG * 4), dtype=torch.float32, device=X.device)
    Xp[:N, :D] = (X.float() - 0.5) / 0.5 if transform else X.float()
    return Xp.view(T, 16, KG, 4).permute(0, 2, 3, 1).reshape(T, KG, 64).contiguous()


def eval_errors_async(X, y, split: int, W, d_in, d_out, transform=True, Xt=None):
    """Error rates of W on rows [0, split) and [split, N) of X from ONE kernel launch and one
    read-back (test error + 1->7 attack rate).  Returns a callable giving (err_a, err_b)."""
    N = X.shape[0]
    na, nb = split, N - split
    if N == 0 or X.device.type != "cuda":
        a = eval_error(X[:split], y[:split], W, d_in, d_out, transform) if na else 0.0
        b = eval_error(X[split:], y[split:], W, d_in, d_out, transform) if nb else 0.0
        return lambda: (a, b)
    # accumulator reset, kernel and read-back in one native call; the download is queued right behind the
    # kernel: the read-back waits for the evaluation only, not for whatever the caller queues on the stream
    # afterwards (the next round's head).  Device and host buffers rotate together (lazy_eval reads the
    # host copy up to a few rounds later).
    host = pinned("eval", (2,), torch.int32, depth=4)
    key = (host.data_ptr(), Xt is not None)   # the two kernels keep their own accumulators: only the tiled one
    err = _EVAL_DEV.get(key)                  # leaves its counters zeroed after a launch
    if err is None:
        # [errors of rows < split, errors of the rest, tiles done]: zero before the first launch, and
        # k_eval_error_t's last tile re-zeroes it when it writes the host copy
        err = _EVAL_DEV[key] = torch.zeros((4,), dtype=torch.int32, device=X.device)
    if Xt is not None:   # cached pre-transformed tiles (k_eval_error_t)
        assert Xt.shape[0] == (N + 15) // 16 and Xt.shape[1] * 4 >= d_in and Xt.shape[2] == 64
        _check(hip().bsc_eval_error_t_rb(_p(Xt), _p(y), N, Xt.shape[1], d_in, d_out, _p(W), int(split), _p(err),
                                         host.data_ptr(), _stream()), "eval_error_t")
    else:
        _check(hip().bsc_eval_error_rb(_p(X), _p(y), N, d_in, d_out, _p(W), int(transform), int(split), _p(err),
                                       host.data_ptr(), _stream()), "eval_error")
    ev = S.record()

    def result():
        S.host_wait(ev)
        e = host.tolist()
        return (e[0] / na if na else 0.0, e[1] / nb if nb else 0.0)
    result.ready = ev.query   # the read-back has landed (result() will not wait)
    return result


def eval_error_async(X, y, W, d_in, d_out, transform=True):
    """Queue the evaluation kernel; returns a zero-argument callable giving the error rate."""
    f = eval_errors_async(X, y, X.shape[0], W, d_in, d_out, transform)
    return lambda: f()[0]


def eval_error(X, y, W, d_in, d_out, transform=True) -> float:
    """1 - accuracy of the softmax model W on (X, y) (client.getTestErr / get17AttackRate)."""
    N = X.shape[0]
    if N == 0:
        return 0.0
    if X.device.type == "cuda":
        return eval_error_async(X, y, W, d_in, d_out, transform)()
    Wm = W.to(torch.float32)
    xb = (X - 0.5) / 0.5 if transform else X
    logits = xb @ Wm[: d_out * d_in].view(d_out, d_in).T + Wm[d_out * d_in:]
    pred = torch.argmax(logits, 1)
    return float((pred != y.long()).sum()) / N


# ---------------------------------------------------------------------------- K12 recovery
def recover(agg_y, xs, poly: int, d: int, W, qscale=1e4):
    """Recover the aggregated quantised update from miner shares and apply it to W.

    agg_y int64 [nchunks, npts]; xs int32 [npts].  Returns (W_new fp64 [d], coeffs int64
    [nchunks, poly], status int32 [nchunks]).
    """
    nchunks, npts = agg_y.shape
    dev = agg_y.device
    W_new = torch.empty_like(W)
    coeffs = torch.empty((nchunks, poly), dtype=torch.int64, device=dev)
    status = torch.empty((nchunks,), dtype=torch.int32, device=dev)
    if dev.type == "cuda":
        _check(hip().bsc_recover(_p(agg_y), nchunks, npts, _p(xs), poly, d, _p(W), float(qscale), _p(W_new),
                                 _p(coeffs), _p(status), _stream()), "recover")
        return W_new, coeffs, status
    from ..native import rt

    xl = [int(v) for v in xs]
    Wn = W.numpy().copy()
    for k in range(nchunks):
        r = rt().recover_exact(xl, [int(v) for v in agg_y[k]], poly - 1)
        status[k] = 1 if r is not None else 0
        r = r if r is not None else [0] * poly
        coeffs[k] = torch.tensor(r, dtype=torch.int64)
        for j in range(poly):
            i = k * poly + j
            if i < d:
                Wn[i] = Wn[i] + float(r[j]) / qscale
    W_new.copy_(torch.from_numpy(Wn))
    return W_new, coeffs, status


def recovery_weights(xs, poly: int) -> dict:
    """Exact integer recovery weights for one x-point layout: the inverse Vandermonde of the `poly`
    basis nodes of smallest |x| (kyber.go:809-857 solves the same system by QR) as A / Dn with
    integer A, Dn = 2^shift * Dodd and Dodd^-1 mod 2^128 -- computed once per miner layout."""
    from fractions import Fraction
    from math import lcm

    xs = [int(x) for x in xs]
    order = sorted(range(len(xs)), key=lambda i: (abs(xs[i]), xs[i]))[:poly]
    nodes = [xs[i] for i in order]
    n = len(nodes)
    M = [[Fraction(x) ** k for k in range(n)] for x in nodes]
    inv = [[Fraction(int(i == j)) for j in range(n)] for i in range(n)]
    for c in range(n):   # Gauss-Jordan over the rationals
        p = next(r for r in range(c, n) if M[r][c] != 0)
        M[c], M[p], inv[c], inv[p] = M[p], M[c], inv[p], inv[c]
        f = M[c][c]
        M[c] = [v / f for v in M[c]]
        inv[c] = [v / f for v in inv[c]]
        for r in range(n):
            if r != c and M[r][c] != 0:
                g = M[r][c]
                M[r] = [a - g * b for a, b in zip(M[r], M[c])]
                inv[r] = [a - g * b for a, b in zip(inv[r], inv[c])]
    Dn = 1
    for row in inv:
        for v in row:
            Dn = lcm(Dn, v.denominator)
    A = [[int(v * Dn) for v in row] for row in inv]
    assert max(abs(a) for r in A for a in r) < 2 ** 40, "recovery weights out of range"
    shift = (Dn & -Dn).bit_length() - 1
    odd = Dn >> shift
    iv = pow(odd, -1, 1 << 128)
    return {"A": np.asarray(A, dtype=np.int64), "basis": order, "shift": shift, "inv_lo": iv & (2 ** 64 - 1),
            "inv_hi": iv >> 64, "Dn": Dn}


def recover_rows(ys, mask, ycols, xs, weights: dict, A_dev, basis_dev, poly: int, d: int, W, qscale=1e4):
    """Fused miner share sums + exact recovery + W update (GPU, k_recover_w).

    ys int64 [R, nch, T] (R = 1 with mask None: already totals); mask int32 [R] or None; ycols /
    xs int32 [npts] (the contributing miners' columns and x-points); weights from recovery_weights
    with A_dev / basis_dev its device copies.  Returns (W_new fp64 [d], coeffs int64 [nch, poly],
    status int32 [nch], agg int64 [nch, npts])."""
    R, nch, T = ys.shape
    npts = ycols.numel()
    dev = ys.device
    W_new = torch.empty_like(W)
    coeffs = torch.empty((nch, poly), dtype=torch.int64, device=dev)
    status = torch.empty((nch,), dtype=torch.int32, device=dev)
    agg = torch.empty((nch, npts), dtype=torch.int64, device=dev)
    if dev.type != "cuda":
        rows = ys if mask is None else ys[mask.bool()]
        agg.copy_(rows.sum(0).index_select(1, ycols.long()))
        W_new, coeffs, status = recover(agg, xs, poly, d, W, qscale)
        return W_new, coeffs, status, agg
    assert ys.dtype == torch.int64 and ys.is_contiguous() and (mask is None or mask.numel() == R)
    _check(hip().bsc_recover_w(_p(ys), R, nch, T, _p(mask), _p(ycols), _p(xs), npts, _p(A_dev), _p(basis_dev), poly,
                               weights["shift"], weights["inv_lo"], weights["inv_hi"], d, _p(W), float(qscale),
                               _p(W_new), _p(coeffs), _p(status), _p(agg), _stream()), "recover_w")
    return W_new, coeffs, status, agg


def sum_rows_i64(ys: torch.Tensor, rows: torch.Tensor | None = None, mask: torch.Tensor | None = None):
    """out[...] = sum over the selected rows r of ys[r, ...] (int64, exact): a rank's partial share-value
    sums of its kept workers (aggregateSecret's Y sums, kyber.go:244-287).  rows: int32 row indices, or
    mask: int32 [R] flags (device-side selection), or neither (every row)."""
    R = ys.shape[0]
    C = ys[0].numel() if R else int(np.prod(ys.shape[1:]))
    out = torch.empty(ys.shape[1:], dtype=torch.int64, device=ys.device)
    if ys.device.type != "cuda":
        sel = ys if rows is None and mask is None else ys[rows.long()] if rows is not None else ys[mask.bool()]
        out.copy_(sel.sum(0))
        return out
    assert ys.dtype == torch.int64 and ys.is_contiguous()
    assert rows is None or (rows.dtype == torch.int32 and rows.is_contiguous())
    assert mask is None or (mask.dtype == torch.int32 and mask.numel() == R)
    nsel = rows.numel() if rows is not None else R
    _check(hip().bsc_sum_rows_i64(_p(ys), R, C, _p(rows), nsel, _p(mask), _p(out), _stream()), "sum_rows_i64")
    return out


def add_rows(delta, rows, W):
    """W + sum of delta[rows] (fp64, sequential like mat.Dense.Add)."""
    D = W.numel()
    if W.device.type == "cuda":
        out = torch.empty_like(W)
        _check(hip().bsc_add_rows(_p(delta), D, _p(rows), rows.numel(), _p(W), _p(out), _stream()), "add_rows")
        return out
    acc = W.clone()
    for r in rows.tolist():
        acc += delta[r].double()
    return acc
