"""Log parser and sweep/bench plumbing on CPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_logparse_reference_format(tmp_path):
    from biscotti_amd.utils.logparse import parse_attack_rates, parse_train_errors, sec_per_round

    lines = [
        "[peer] 23:59:58.500000 honest.go:153: 3:Train Error is 0.61667 in Iteration 0\n",
        "[peer] 23:59:58.600000 honest.go:153: 4:Train Error is 0.61667 in Iteration 0\n",  # second peer: ignored
        "[peer] 23:59:59.000000 honest.go:155: 3:Attack Rate is 0.50000 in Iteration 0\n",
        "[peer] 00:00:00.500000 honest.go:153: 3:Train Error is 0.52167 in Iteration 1\n",  # past midnight
        "noise\n",
    ]
    rows = parse_train_errors(lines)
    assert [(r[0], r[1]) for r in rows] == [(0, 0.61667), (1, 0.52167)]
    assert abs(sec_per_round(rows) - 2.0) < 1e-9
    assert parse_attack_rates(lines) == {0: 0.5}


def test_engine_log_lines_parse(tmp_path):
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine
    from biscotti_amd.utils.logparse import parse_train_errors, phase_breakdown

    trace = tmp_path / "t.jsonl"
    log_dir = tmp_path / "logs"
    log_dir.mkdir()
    eng = BiscottiEngine(RunConfig(num_nodes=5, dataset="creditcard", num_verifiers=1, num_miners=2,
                                   num_noisers=1, device="cpu", log_dir=str(log_dir), trace_file=str(trace)))
    for _ in range(3):
        eng.run_round()
    eng.close()
    logs = list(log_dir.iterdir())
    assert logs
    rows = parse_train_errors(open(logs[0]).readlines())
    assert [r[0] for r in rows] == [0, 1, 2]
    pb = phase_breakdown(str(trace))
    assert pb["rounds"] == 3 and "verify" in pb


def test_bench_cpu_credit4_and_set_override():
    out = subprocess.run([sys.executable, "bench.py", "--config", "credit4", "--steps", "3", "--warmup", "1",
                          "--set", "seed=7"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(next(ln for ln in out.stdout.splitlines() if ln.startswith("{")))
    assert rec["config"]["name"] == "credit4" and rec["chain_valid"] and rec["steps"] == 3
    for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
              "dtype", "data", "config"):
        assert k in rec


def test_sandbox_models_train_on_cpu():
    from biscotti_amd.sandbox import run

    r = run("softmax", "creditcard", clients=4, iters=150, eval_every=50, lr=1e-2, device="cpu", verbose=False)
    assert r["final_test_error"] < r["history"][0]["test_error"] + 1e-9
    for model, ds in [("cifar_cnn", "cifar"), ("lfw_cnn", "lfw")]:
        r = run(model, ds, clients=2, iters=60, eval_every=30, lr=5e-3, device="cpu", verbose=False)
        assert r["final_test_error"] <= r["history"][0]["test_error"] + 0.05
        assert len(r["history"]) == 3


def test_sandbox_cnn_architectures_match_reference():
    """Layer shapes and parameter counts of lfw_cnn_model.py / cifar_cnn_model.py / mnist_cnn_model.py."""
    import torch

    from biscotti_amd.models import zoo as Z

    lfw = Z.LFWCNNModel()
    assert [tuple(p.shape) for p in lfw.parameters()] == [(18, 3, 3, 3), (18,), (36, 18, 3, 3), (36,), (2, 5940), (2,)]
    assert sum(p.numel() for p in lfw.parameters()) == 18254          # datasets.get_num_params('lfw')
    assert lfw(torch.zeros(2, 3 * 62 * 47)).shape == (2, 2)
    cifar = Z.CIFARCNNModel()
    assert [tuple(p.shape) for p in cifar.parameters()] == [(20, 3, 3, 3), (20,), (10, 25920), (10,)]
    assert sum(p.numel() for p in cifar.parameters()) == 540 + 20 + 259200 + 10
    assert cifar(torch.zeros(2, 3 * 32 * 32)).shape == (2, 10)
    mnist = Z.MNISTCNNModel()
    assert mnist(torch.zeros(2, 784)).shape == (2, 10)


def test_native_selftest_under_asan_ubsan():
    """Host runtime under AddressSanitizer + UBSan, 6 threads (race/sanitizer coverage)."""
    r = subprocess.run([sys.executable, "-m", "biscotti_amd._build", "--sanitize"], cwd=ROOT, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "selftest: ok" in r.stdout


def test_native_pool_under_tsan():
    """The thread pool and job dispatcher the bindings run their VRF / Schnorr / KZG batches on, under
    ThreadSanitizer: overlapping pool jobs from 6 submitting threads, dispatcher tasks that run pool jobs and wait
    on an earlier task (SURVEY §5 race detection; the reference has none)."""
    r = subprocess.run([sys.executable, "-m", "biscotti_amd._build", "--tsan"], cwd=ROOT, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "selftest pool: ok" in r.stdout
    assert "ThreadSanitizer" not in r.stderr


def test_centralblock_prototype():
    import numpy as np

    from biscotti_amd.centralblock import CentralBlock, invert

    cb = CentralBlock(n_branches=2, poisoners=2, batch=20, device="cpu")
    e0 = cb.evaluate()["best_test_error"]
    for _ in range(30):
        cb.step()
    assert all(sum(h) == len(cb.clients) for h in cb.history)      # every client submits once per step
    assert cb.evaluate()["best_test_error"] < e0
    img = invert(np.arange(7840, dtype=np.float64))
    assert img.shape == (784,) and abs(img.max() - 2.55 * 1567 / 7839) < 1e-12


def test_eval_plotters(tmp_path):
    """The figure set of the reference's eval scripts from this framework's own traces / bench lines."""
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine
    from biscotti_amd.protocol.fedsys import FedSysEngine
    from biscotti_amd.utils import plots

    tr, ftr = tmp_path / "b.jsonl", tmp_path / "f.jsonl"
    kw = dict(num_nodes=6, dataset="creditcard", num_verifiers=1, num_miners=2, num_noisers=1, noising=False,
              device="cpu", seed=2)
    eng = BiscottiEngine(RunConfig(trace_file=str(tr), **kw))
    for _ in range(4):
        eng.run_round()
    eng.close()
    fed = FedSysEngine(RunConfig(trace_file=str(ftr), **kw))
    for _ in range(4):
        fed.run_round()
    ref = os.path.join(ROOT, "profiles", "reference_curves.json")
    outs = [plots.convergence(str(tr), str(ftr), str(tmp_path / "c.pdf"), ref),
            plots.poisoning(str(tr), str(tmp_path / "p.pdf"), ref),
            plots.breakdown(str(tr), str(tmp_path / "k.pdf"), skip=1)]
    bl = []
    for n in (4, 6):
        f = tmp_path / f"bench{n}.txt"
        f.write_text(json.dumps({"value": 0.001 * n, "n_gpus": 1, "config": {"peers": n}}) + "\n")
        bl.append(str(f))
    outs.append(plots.scaling(bl, "peers", str(tmp_path / "s.pdf")))
    hm = tmp_path / "poison_ns.jsonl"
    hm.write_text("".join(json.dumps({"attack_rate_last10_mean": 0.1 * i + 0.01 * j,
                                      "config": {"poisoning": po, "ns_percent": ns}}) + "\n"
                          for i, po in enumerate((0.1, 0.3, 0.5)) for j, ns in enumerate((20, 40, 70))))
    outs.append(plots.heatmap([str(hm)], str(tmp_path / "h.pdf")))
    assert all(os.path.getsize(o) > 1000 for o in outs)


def test_vrf_security_models_and_lottery(tmp_path):
    """eval_vrf_security / eval_privacy_noise_attack models; the capture probability of this
    framework's own lottery (distinct stake-weighted picks) matches the hypergeometric model."""
    from biscotti_amd.native import rt
    from biscotti_amd.utils import vrf_security as V

    assert abs(V.majority_capture_prob(3, 0.5) - 0.5) < 1e-12
    assert V.min_committee_size(0.1, 0.001) == 8      # binomial tail (even sizes need a strict majority of c/2 + 1)
    assert V.noise_attack_prob_reference(0.3, 2, 3) == 0.3 ** 2 * (1 - 0.3 ** 3)
    trials = 1500
    emp = V.simulate_verifier_capture(rt(), 30, 30, 3, trials)
    model = V.majority_capture_prob_distinct(30, 9, 3)
    sd = (model * (1 - model) / trials) ** 0.5
    assert abs(emp - model) < 4 * sd + 0.01, (emp, model)
    assert (tmp_path / "c.pdf").exists() is False
    V.plot_committee(str(tmp_path / "c.pdf"))
    V.plot_noise(str(tmp_path / "n.pdf"))
    assert (tmp_path / "c.pdf").stat().st_size > 0 and (tmp_path / "n.pdf").stat().st_size > 0


def test_bench_scale_weak_preset_four_gloo_ranks():
    """bench.py --config scale_weak on 4 gloo ranks (torchrun on 127.0.0.1): 100 peers per rank -> a 400-peer job
    (creditcard keeps the CPU crypto cheap); the JSON names the job's peers and the per-rank packing, and the chain
    verifies on every rank."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
                          "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", "4",
                          "--config", "scale_weak", "--steps", "2", "--warmup", "1", "--rounds", "3",
                          "--set", "dataset=creditcard", "--set", "noising=false", "--set", "host_threads=2"],
                         cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads(next(ln for ln in out.stdout.splitlines() if ln.startswith("{")))
    assert rec["config"]["name"] == "scale_weak" and rec["config"]["peers"] == 400 and rec["n_gpus"] == 4
    assert rec["config"]["parallelism"].startswith("dp4") and "100/GPU" in rec["config"]["parallelism"]
    assert rec["chain_valid"] and len(rec["per_rank"]) == 4
    assert rec["contributors_per_block"] > 0 and rec["stake_initial"] == 4000
