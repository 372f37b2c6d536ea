"""Multi-process runs over gloo (CPU): every rank must hold the same chain, and it must equal the
single-process chain byte for byte (deterministic timestamps) -- the localTest.sh oracle."""
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kw, rounds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    count = kw.pop("_count_collectives", False)
    comm = Comm.init(device="cpu")
    eng = BiscottiEngine(RunConfig(**kw), comm)
    calls, reads = [], []
    if count:
        import torch.distributed as dist

        def wrap(name):
            real = getattr(dist, name)

            def counting(*a, **k):
                calls.append(name)
                return real(*a, **k)
            setattr(dist, name, counting)
        for name in ("all_gather_into_tensor", "all_gather", "all_reduce", "broadcast", "all_to_all_single",
                     "all_to_all", "reduce_scatter_tensor", "gather", "scatter", "all_gather_object",
                     "broadcast_object_list", "reduce"):
            wrap(name)
        real_d2h = eng._d2h_async

        def counting_d2h(*ts):
            reads.append(len(ts))
            return real_d2h(*ts)
        eng._d2h_async = counting_d2h
    per_round = []
    for _ in range(rounds):
        n0, r0 = len(calls), len(reads)
        r = eng.run_round()
        per_round.append((len(calls) - n0, len(reads) - r0, r.empty))
    if count:
        # every non-empty secure round after the first (whose head is opened inside it): the noise-aware
        # Gram's delta gather (the next round's head), the gather of commitments + noiser ids after the
        # VRF outputs and the aggregation gather -- 2 without the noise-aware Krum -- and one batched
        # read-back of the recovered model (+ clocks); nothing else crosses ranks
        want = 3 if eng._noise_krum() else 2
        assert all(c == want and rd <= 2 for c, rd, empty in per_round[1:] if not empty), (want, per_round)
        assert any(not empty for *_, empty in per_round)
        # each rank computes the VRF outputs of the peers it hosts only (heads of rounds + 1)
        assert eng.stats["vrf_outputs"] <= (rounds + 1) * len(eng.local), (eng.stats["vrf_outputs"], len(eng.local))
    q.put((rank, [bytes(eng.fsm.chain.block(i).hash) for i in range(len(eng.fsm.chain))]))
    comm.barrier()
    comm.shutdown()


def _run(world, kw, rounds):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kw, rounds, q)) for r in range(world)]
    import queue
    import time

    for p in ps:
        p.start()
    out, deadline = {}, time.time() + 600
    try:
        while len(out) < world:
            try:
                r, hashes = q.get(timeout=1.0)
                out[r] = hashes
            except queue.Empty:
                if any(p.exitcode not in (None, 0) for p in ps) or time.time() > deadline:
                    raise AssertionError("a rank failed: " + str([p.exitcode for p in ps]))
        for p in ps:
            p.join(timeout=120)
            assert p.exitcode == 0
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
    return out


KW = dict(num_nodes=6, dataset="creditcard", num_verifiers=2, num_miners=3, num_noisers=1, epsilon=1.0,
          device="cpu", seed=11, deterministic_time=True)


@pytest.mark.parametrize("secure_agg", [True, False])
def test_two_ranks_match_single_process(secure_agg):
    kw = dict(KW, secure_agg=secure_agg)
    single = _run(1, kw, 4)[0]
    multi = _run(2, kw, 4)
    assert multi[0] == multi[1]
    assert multi[0] == single


def test_three_ranks_uneven_packing():
    kw = dict(KW, num_nodes=7)
    single = _run(1, kw, 3)[0]
    multi = _run(3, kw, 3)
    assert multi[0] == multi[1] == multi[2]
    assert multi[0] == single


@pytest.mark.parametrize("world,noising", [(2, True), (4, True), (8, True), (3, False)])
def test_collectives_per_round(world, noising):
    """A secure-aggregation round with Multi-Krum issues a fixed number of collectives of any kind on 2-8
    ranks (3 with the noise-aware Krum: delta gather, commitments + noiser ids, aggregation; 2 without)
    and at most two batched read-backs: no accept-mask, share, signature or block traffic (every rank
    replicates the committee and the recovery).  Every rank proves only its own peers' VRF outputs, and
    all ranks hold the single-process chain."""
    kw = dict(KW, num_nodes=9, seed=3, noising=noising)
    single = _run(1, kw, 3)[0]
    out = _run(world, dict(kw, _count_collectives=True), 3)
    assert all(out[r] == single for r in range(world))


def test_mnist_noise_aware_krum_ranks_match_single_process():
    """MNIST with the noise-aware committee Krum (Gram over [deltas; noise vectors] on the flat peer layout,
    noiser ids gathered): 1 rank and 3 ranks give the same chain, poisoners included."""
    kw = dict(num_nodes=8, dataset="mnist", num_verifiers=2, num_miners=2, num_noisers=2, epsilon=1.0,
              device="cpu", seed=4, deterministic_time=True, poisoning=0.25)
    single = _run(1, kw, 3)[0]
    multi = _run(3, kw, 3)
    assert multi[0] == multi[1] == multi[2] == single


def test_peer_processes_localtest_oracle():
    """DistSys/localTest.sh: N processes `peer -i k -t N -d creditcard`, identical chain dumps."""
    n = 4
    port = _free_port()
    env = dict(os.environ, MASTER_PORT=str(port), PYTHONPATH=ROOT)
    procs = [subprocess.Popen([sys.executable, "-m", "biscotti_amd.peer", f"-i={k}", f"-t={n}", "-d=creditcard",
                               "-na=1", "-nv=1", "-nn=1", "-np=false", "--device", "cpu", "--rounds", "3",
                               "--print-chain", "all", "--deterministic-time"],
                              cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
             for k in range(n)]
    outs = [b"\n".join(ln for ln in p.communicate(timeout=600)[0].split(b"\n") if not ln.startswith(b"[Gloo]"))
            for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert all(o == outs[0] for o in outs) and outs[0].count(b"Hash: ") == 4
