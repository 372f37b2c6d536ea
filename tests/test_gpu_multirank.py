"""Multi-rank engine on the GPU: 2 and 4 ranks share cuda:0 over the gloo backend, and 2 ranks over
RCCL (distinct NCCL_HOSTIDs: RCCL's socket transport on loopback), which runs every device-side
multi-rank path -- the all_gather of
commitments + noised deltas, the replicated committee Krum, per-rank partial share sums and their
all_gather, replicated exact recovery -- and must reproduce the single-process GPU chain byte for
byte (deterministic timestamps), also with poisoners and churn."""
import os
import queue
import sys
import time

import pytest
import torch.multiprocessing as mp

from test_distributed_cpu import ROOT, _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, kw, rounds, q, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", BSC_TABLE_B0="10")
    if backend == "nccl":
        # RCCL refuses two ranks on one device within a host; a distinct host id per rank makes it
        # connect them through its socket transport on loopback -- RCCL's init, proxy threads and
        # collective kernels all run, on cuda:0 for both ranks
        os.environ.update(NCCL_HOSTID=f"biscotti-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    sys.path.insert(0, ROOT)
    import torch

    from biscotti_amd.parallel.comm import Comm
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    comm = Comm.init(backend=backend) if world > 1 else Comm(device=torch.device("cuda", 0))
    assert comm.device.type == "cuda"
    assert world == 1 or comm.backend == backend, (comm.backend, backend)
    eng = BiscottiEngine(RunConfig(**kw), comm)
    for _ in range(rounds):
        eng.run_round()
    stats = {k: v for k, v in eng.stats.items() if isinstance(v, (int, float))}
    q.put((rank, ([bytes(eng.fsm.chain.block(i).hash) for i in range(len(eng.fsm.chain))], stats)))
    comm.barrier()
    eng.close()
    comm.shutdown()


def _run(world, kw, rounds, backend="gloo"):
    """rank -> chain hashes (every rank must agree)."""
    return {r: h for r, (h, _) in _run_stats(world, kw, rounds, backend).items()}


def _run_stats(world, kw, rounds, backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kw, rounds, q, backend)) for r in range(world)]
    for p in ps:
        p.start()
    out, deadline = {}, time.time() + 400
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


@pytest.mark.parametrize("secure_agg", [True, False])
def test_gpu_two_ranks_match_single_process(secure_agg):
    kw = dict(num_nodes=12, dataset="mnist", seed=5, deterministic_time=True, secure_agg=secure_agg,
              max_iterations=100)
    single = _run(1, kw, 3)[0]
    multi = _run(2, kw, 3)
    assert multi[0] == multi[1]
    assert multi[0] == single


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_gpu_four_ranks_poisoning_and_churn_match_single_process(backend):
    """4 ranks with poisoners and churn, over gloo and over RCCL (socket transport between the ranks
    sharing cuda:0): every device-side multi-rank path -- the pre-step's delta gather and noise-aware
    Gram, the commitments + noiser-ids gather, the per-rank share sums and their gather, the replicated
    recovery -- must give the single-process chain byte for byte."""
    kw = dict(num_nodes=16, dataset="mnist", seed=9, deterministic_time=True, max_iterations=100, poisoning=0.3,
              churn=0.1, num_verifiers=3)
    single = _run(1, kw, 4)[0]
    multi = _run(4, kw, 4, backend=backend)
    assert multi[0] == multi[1] == multi[2] == multi[3]
    assert multi[0] == single


def test_gpu_two_ranks_over_rccl_match_single_process():
    """The same round over the RCCL ("nccl") backend: both collectives of a secure round (the
    packed all_gathers) run through RCCL and the chain equals the single-process GPU chain."""
    kw = dict(num_nodes=12, dataset="mnist", seed=5, deterministic_time=True, max_iterations=100)
    single = _run(1, kw, 3)[0]
    multi = _run(2, kw, 3, backend="nccl")
    assert multi[0] == multi[1]
    assert multi[0] == single


@pytest.mark.parametrize("world,extra", [(2, ""), (4, ",multi_spec_front"), (2, ",multi_spec_front"),
                                         (4, ",multi_early_front")])
def test_gpu_one_rank_per_gpu_fast_path_over_rccl(world, extra):
    """The configuration an 8-GPU node runs (one rank per GPU): the speculative next-round head forced on
    (ablation spec_head_shared; it is off by default only because these ranks share cuda:0), the native pre-step
    (local step + chunk commitments), the Gram's tiles split across ranks, the native multi-rank
    aggregation (partial sums -> one packed all_gather -> recovery), the next round's front launched before the
    block's commit on every rank (multi_spec_front: the speculative front, its collectives in the same order
    everywhere), at the commit (multi_early_front) or at the round's start (default).  Every rank must use every fast path
    in every round after the first, and the chain must equal one process's byte for byte."""
    rounds = 6
    kw = dict(num_nodes=20, dataset="mnist", seed=13, deterministic_time=True, max_iterations=100,
              ablation="spec_head_shared")
    single, s1 = _run_stats(1, kw, rounds)[0]
    out = _run_stats(world, dict(kw, ablation=kw["ablation"] + extra), rounds, backend="nccl")
    for r in range(world):
        hashes, st = out[r]
        assert hashes == single, f"rank {r} chain differs"
        for k in ("pre_steps", "spec_head", "device_aggregations", "early_vrf"):
            assert st.get(k, 0) >= rounds - 1, (r, k, st)
        assert st.get("spec_misses", 0) == 0 and st.get("audit_failures", 0) == 0, st
        assert st.get("native_collectives") == 1, (r, st)
        if "multi_spec_front" in extra:   # launched before the commit and adopted, on every rank
            assert st.get("spec_fronts", 0) >= rounds - 2 and "spec_front_drops" not in st, (r, st)
        else:
            assert "spec_fronts" not in st, (r, st)
        if extra:
            assert st.get("early_fronts", 0) >= rounds - 2, (r, st)
    assert s1.get("spec_head", 0) >= rounds - 1, s1


def test_gpu_rank_without_candidate_rows_keeps_the_chain():
    """4 RCCL ranks of 5 peers with the speculative horizon at the leader's cap (spec_tight): some rank has no
    candidate row within the horizon in some round and keeps the successor plan with no MSM to launch (the same
    speculative-head decision as its peers: the Krum tables, the candidate set and the collectives stay the
    same everywhere); misses are topped up on the host path; the chain equals one process's byte for byte."""
    rounds = 10
    kw = dict(num_nodes=20, dataset="mnist", seed=23, deterministic_time=True, max_iterations=100,
              ablation="spec_head_shared,spec_tight")
    single, s1 = _run_stats(1, kw, rounds)[0]
    out = _run_stats(4, kw, rounds, backend="nccl")
    for r in range(4):
        hashes, st = out[r]
        assert hashes == single, f"rank {r} chain differs"
        assert st.get("spec_head", 0) >= rounds - 1 and st.get("audit_failures", 0) == 0, (r, st)
    assert len({out[r][1].get("spec_misses", 0) for r in range(4)}) == 1   # the same top-up decisions
    no_rows = [out[r][1].get("spec_head_no_rows", 0) for r in range(4)]
    assert sum(no_rows) >= 1, no_rows   # (deterministic: rank 1 has one such round)


def test_gpu_spec_horizon_two_ranks_100_peers_over_rccl():
    """The headline size (100 peers) on two RCCL ranks with the speculative head forced on: after 8 blocks
    the speculative MSM covers only the candidates up to the replicated horizon (head.py SPEC_MARGIN), every
    rank takes the same fast / top-up decisions, and the chain equals one process's byte for byte."""
    rounds = 12
    kw = dict(num_nodes=100, dataset="mnist", seed=17, deterministic_time=True, max_iterations=100,
              ablation="spec_head_shared")
    single, s1 = _run_stats(1, kw, rounds)[0]
    out = _run_stats(2, kw, rounds, backend="nccl")
    for r in range(2):
        hashes, st = out[r]
        assert hashes == single, f"rank {r} chain differs"
        assert st.get("spec_head", 0) >= rounds - 1 and st.get("audit_failures", 0) == 0, (r, st)
    assert out[0][1].get("spec_misses", 0) == out[1][1].get("spec_misses", 0) == s1.get("spec_misses", 0)
    # each rank launches its own peers' rows: together the single process's rows
    assert out[0][1]["spec_rows"] + out[1][1]["spec_rows"] == s1["spec_rows"], (out[0][1], out[1][1], s1)


def test_gpu_eight_ranks_100_peers_over_rccl():
    """The job an 8-GPU node runs at the headline size, rehearsed with 8 RCCL ranks sharing cuda:0: 100 peers
    split 12/13 per rank, the speculative head forced on, every fast path on every rank in every round after the
    first, no audit failure, and the chain equal to one process's byte for byte (the localTest.sh oracle,
    DistSys/localTest.sh:47-87)."""
    rounds = 6
    kw = dict(num_nodes=100, dataset="mnist", seed=19, deterministic_time=True, max_iterations=100,
              ablation="spec_head_shared", host_threads=2)
    single, s1 = _run_stats(1, kw, rounds)[0]
    out = _run_stats(8, kw, rounds, backend="nccl")
    for r in range(8):
        hashes, st = out[r]
        assert hashes == single, f"rank {r} chain differs"
        for k in ("pre_steps", "spec_head", "early_vrf"):
            assert st.get(k, 0) >= rounds - 1, (r, k, st)
        assert st.get("device_aggregations", 0) + st.get("spec_misses", 0) >= rounds - 1, (r, st)
        assert st.get("audit_failures", 0) == 0, (r, st)
        assert st.get("native_collectives") == 1, (r, st)   # the round's own RCCL communicator ran
    assert sum(out[r][1]["spec_rows"] for r in range(8)) == s1["spec_rows"]


def test_gpu_emulated_rank0_native_collectives():
    """bench.py --emulate-world N: rank 0 of an N-rank job alone on the GPU -- its peers' work, the native fused calls
    with every collective replaced by ONE replicate launch (rank 0's contribution in every slot) -- runs the multi-rank
    fast paths (native collectives, packed verification row, the aggregation + next Gram in one call) and keeps a valid
    chain."""
    import subprocess
    import json

    out = subprocess.run([sys.executable, "bench.py", "--emulate-world", "4", "--steps", "4", "--warmup", "2",
                          "--rounds", "8", "--peers", "24"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads(next(ln for ln in out.stdout.splitlines() if ln.startswith("{")))
    st = rec["engine_stats"]
    assert rec["emulated_world"] == 4 and rec["chain_valid"], rec
    assert st["native_collectives"] == 1 and st.get("pre_steps", 0) >= 4 and st.get("device_aggregations", 0) >= 4, st
    assert st["audit_failures"] == 0, st
