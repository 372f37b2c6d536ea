"""Aggregate commitment audit, crash-tolerant chain files and rank-failure restarts (CPU)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from biscotti_amd.protocol.config import RunConfig
from biscotti_amd.protocol.engine import BiscottiEngine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(**kw):
    base = dict(num_nodes=6, dataset="creditcard", num_verifiers=1, num_miners=3, num_noisers=1, noising=False,
                device="cpu", seed=7, deterministic_time=True)
    base.update(kw)
    return RunConfig(**base)


def test_audit_accepts_honest_aggregate():
    eng = BiscottiEngine(_cfg())
    res = [eng.run_round() for _ in range(3)]
    assert all(not r.empty for r in res)
    assert eng.stats["audit_failures"] == 0


def test_audit_check_matches_host_commitments(rt):
    """check_aggregate: ok iff a miner's summed chunk commitment commits to the recovered chunk."""
    eng = BiscottiEngine(_cfg())
    cr = eng.crypto
    rng = np.random.default_rng(1)
    coeffs = torch.from_numpy(rng.integers(-10**6, 10**6, size=(cr.nchunks, cr.poly)))
    good = np.stack([np.frombuffer(cr.key.commit(np.ascontiguousarray(coeffs[k, :min(cr.poly, cr.d - k * cr.poly)]
                                                                      .numpy()), k * cr.poly), np.uint8)
                     for k in range(cr.nchunks)])
    bad = good.copy()
    bad[1] = np.frombuffer(rt.g1_generator(), np.uint8)
    ok = cr.check_aggregate(coeffs, torch.from_numpy(np.stack([good, bad])))
    assert ok[0].all()
    assert ok[1, 1] == 0 and ok[1].sum() == cr.nchunks - 1


def test_audit_rejects_tampered_recovery(monkeypatch):
    """A recovered update that the miners' commitments do not cover is refused: empty block."""
    from biscotti_amd.protocol import engine as E

    real = E.K.recover

    def tampered(agg, xs, poly, d, W, qscale):
        W_new, coeffs, status = real(agg, xs, poly, d, W, qscale)
        coeffs[0, 0] += 1
        W_new[0] += 1.0 / qscale
        return W_new, coeffs, status
    monkeypatch.setattr(E.K, "recover", tampered)
    eng = BiscottiEngine(_cfg())
    r = eng.run_round()
    assert r.empty and eng.stats["audit_failures"] == 1
    assert eng.fsm.chain.verify()[0]


def test_chain_file_with_torn_tail_resumes(tmp_path):
    path = str(tmp_path / "chain.bin")
    a = BiscottiEngine(_cfg(chain_file=path))
    for _ in range(3):
        a.run_round()
    h2 = a.fsm.chain.latest().hash   # iteration 2 (genesis + 3 blocks)
    # a crash in the middle of appending block 3: its record is cut short
    size = os.path.getsize(path)
    a.run_round()
    with open(path, "r+b") as f:
        f.truncate(size + (os.path.getsize(path) - size) // 2)
    b = BiscottiEngine(_cfg(chain_file=path, resume=True))
    assert len(b.fsm.chain) == 4 and b.fsm.chain.latest().hash == h2
    r = b.run_round()
    assert r.iteration == 3 and b.fsm.chain.verify()[0]
    assert os.path.getsize(path) > size   # the torn record was replaced by the new block


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rank_failure_restarts_from_chain_file(tmp_path):
    """Rank 1 dies after committing iteration 2; torchrun restarts the job, which resumes from the
    chain file and finishes the run: every block verifies and no iteration is missing."""
    chain = tmp_path / "chain.bin"
    logs = tmp_path / "logs"
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--max-restarts=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "biscotti_amd.peer",
           "-t=6", "-d=creditcard", "-na=2", "-nv=1", "-nn=1", "-np=false", "--device", "cpu",
           "--max-iterations", "5", "--chain-file", str(chain), "--resume", "--fail-at", "2", "--fail-rank", "1",
           "--deterministic-time", "--comm-timeout", "60", "--print-chain", "rank0"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, "\n".join(l for l in p.stderr.splitlines() if "Train Error" not in l)[-6000:]
    assert "fault injection: rank 1 exits after iteration 2" in p.stderr
    assert "Resumed chain" in p.stderr
    from biscotti_amd.native import rt

    c = rt().Blockchain.load(str(chain))
    assert c.verify()[0]
    its = [c.block(i).data.iteration for i in range(len(c))]
    assert its == list(range(-1, len(c) - 1)) and its[-1] >= 5


def test_native_secagg_model_ring_never_aliases_the_live_model():
    """NativeSecAgg's recovered-model ring (kernels/round.hip bsc_ring_pick, host code: runs without a GPU):
    aggregates computed and then dropped (speculative misses, failed audits, empty blocks) keep the engine's W
    unchanged for several rounds; the next model must never land in W's buffer nor in one of the last two
    results (a queued pre-step may still read it)."""
    import ctypes

    from biscotti_amd.native import hip

    lib = hip()
    ring = (ctypes.c_void_p * 4)(0x1000, 0x2000, 0x3000, 0x4000)
    k, recent = ctypes.c_int(0), (ctypes.c_void_p * 2)()

    def pick(W):
        j = lib.bsc_ring_pick(ring, 4, ctypes.byref(k), W, recent)
        assert j >= 0
        return ring[j]
    W = ring[1]                       # the live model sits in a ring slot (adopted earlier)
    last = []
    for _ in range(12):               # twelve dropped aggregates in a row
        out = pick(W)
        assert out != W and out not in last[-2:]
        last.append(out)
    W = pick(W)                       # adopted: becomes the live model
    for _ in range(6):
        out = pick(W)
        assert out != W
        W = out
