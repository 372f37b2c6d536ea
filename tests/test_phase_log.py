"""--phase-log: the reference's role and phase lines (main.go:332,510-512,1405,1516,1550,1563,1692) let its own
breakdown (eval/eval_performance/parseLogs.py:79-194, ported in utils/logparse.py) rebuild the noising,
verification and secure-aggregation times -- equal to the phase timer's (the JSONL trace) within timer
resolution."""
import json

from biscotti_amd.protocol.config import RunConfig
from biscotti_amd.protocol.engine import BiscottiEngine
from biscotti_amd.utils import logparse as L


def test_phase_log_lines_parse_into_the_trace_phases(tmp_path):
    cfg = RunConfig(num_nodes=8, dataset="creditcard", num_verifiers=2, num_miners=2, num_noisers=1, device="cpu",
                    phase_log=True, log_dir=str(tmp_path), trace_file=str(tmp_path / "trace.jsonl"),
                    deterministic_time=True)
    eng = BiscottiEngine(cfg)
    res = [eng.run_round() for _ in range(10)]
    eng.close()
    lines = [ln.rstrip("\n") for ln in open(tmp_path / "log_0_8.log")]
    trace = [json.loads(ln) for ln in open(tmp_path / "trace.jsonl")]
    assert [t["iteration"] for t in trace] == [r.iteration for r in res]
    # peer 0 sends an update (and logs the worker lines) only in rounds where it is no committee member
    worker = [t for t, r in zip(trace, res) if 0 not in r.verifiers and 0 not in r.miners]
    assert len(worker) >= 3
    verif = L.parse_verif(lines)
    assert len(verif) == len(worker)
    # the log line is written next to the timer's reading, not at the same instant: a preempted thread (xdist
    # workers on a loaded CPU) puts tens of us between them
    for got, t in zip(verif, worker):
        assert abs(got - t["t_verify"]) < 5e-4, (got, t["t_verify"])
    noise = L.parse_noise(lines)
    assert len(noise) == len(worker)
    for got, t in zip(noise, worker):
        assert abs(got - t["t_noise"]) < 5e-4, (got, t["t_noise"])
    aggr = L.parse_aggr(lines)
    assert [k for k, _ in aggr] == list(range(10))
    for (k, got), t in zip(aggr, trace):
        want = t.get("t_shares", 0.0) + t.get("t_recover", 0.0) + t["t_block"]
        # the log's span also covers the host work between those phases (a few ms more on a loaded CPU)
        assert got is not None and want - 1e-3 <= got <= 1.1 * want + 5e-3, (k, got, want)
    # the reference parser's fixed offset (parseLogs.py:184: line[48:len(line)-1]) reads the miner ids
    miners_lines = [ln for ln in lines if "Miners are" in ln]
    assert [[int(x) for x in ln[48:len(ln) - 1].split(" ")] for ln in miners_lines] == [list(r.miners) for r in res]
    # one rank: the leader's aggregation lines also land in its own log file, where parseLogs.py reads them
    for r in res:
        if r.miners and max(r.miners) != 0:
            own = open(tmp_path / f"log_{max(r.miners)}_8.log").read()
            assert f"Got share for {r.iteration}, I am at {r.iteration}" in own
    cols = L.phase_columns(lines)
    assert cols["rounds"] == 10 and cols["verification"] > 0 and cols["sec_agg"] > 0


def test_phase_log_off_writes_no_phase_lines(tmp_path):
    cfg = RunConfig(num_nodes=6, dataset="creditcard", num_verifiers=2, num_miners=2, num_noisers=1, device="cpu",
                    log_dir=str(tmp_path), deterministic_time=True)
    eng = BiscottiEngine(cfg)
    eng.run_round()
    eng.close()
    txt = open(tmp_path / "log_0_6.log").read()
    assert "Train Error" in txt and "Miners are" not in txt and "Sending update" not in txt
