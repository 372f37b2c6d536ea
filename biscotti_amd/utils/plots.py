"""Evaluation figures, the counterparts of the reference's plotting scripts.

  convergence   test error vs training iteration and vs wall time, Biscotti vs FedSys
                (nsdi-eval/scaleup/baselines.py:43-118 -> eval_convrate{,_time}.pdf)
  poisoning     test error and 1->7 attack rate vs iteration for poisoned runs
                (eval/eval_poison/generateResults.py, nsdi-eval/credit/plot_poison.py)
  breakdown     stacked per-phase time per round (usenix-eval/generateResults.py,
                nsdi-eval/increments -> eval_cost_breakdown.pdf)
  scaling       seconds per round vs peers or vs GPUs (nsdi-eval/increments/plot_incremental.py)
  heatmap       attack rate over poisoner fraction x % of updates collected
                (eval/eval_poison_nsamples/plotHeatMap.py)

Inputs are what this framework writes: peer logs in the reference's line format (parsed with
utils.logparse), the engine's JSONL trace (``--trace-file``: per-round error, attack rate, wall time
and phase times), and bench.py result lines.  The reference's own curves (recovered from its PDFs,
profiles/reference_curves.json) can be overlaid as dashed lines.

    python -m biscotti_amd.utils.plots convergence --trace run.jsonl --fedsys-trace fed.jsonl -o conv.pdf
    python -m biscotti_amd.utils.plots poisoning --trace po30.jsonl --reference profiles/reference_curves.json
    python -m biscotti_amd.utils.plots breakdown --trace run.jsonl -o breakdown.pdf
    python -m biscotti_amd.utils.plots scaling --bench a.json b.json ... --x peers -o scaling.pdf
"""
from __future__ import annotations

import argparse
import json
import sys


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def read_trace(path: str) -> list[dict]:
    rows = []
    with open(path) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{"):
                rows.append(json.loads(ln))
    return rows


def read_bench(path: str) -> dict:
    with open(path) as f:
        for ln in reversed(f.read().splitlines()):
            if ln.startswith("{"):
                return json.loads(ln)
    raise ValueError(f"{path}: no bench result line")


def _reference_series(ref_path: str | None, name_part: str, label_part: str):
    if not ref_path:
        return None
    ref = json.load(open(ref_path))
    for f, r in ref.items():
        if name_part in f:
            for s in r.get("series", []):
                if label_part in (s.get("label") or ""):
                    return s
    return None


def _style(ax, xlabel, ylabel, ylim=(0, 1)):
    ax.set_xlabel(xlabel, fontsize=14)
    ax.set_ylabel(ylabel, fontsize=14)
    if ylim:
        ax.set_ylim(*ylim)
    ax.spines["right"].set_visible(False)
    ax.spines["top"].set_visible(False)
    ax.legend(fontsize=11)


def convergence(trace: str, fedsys_trace: str | None = None, out: str = "eval_convrate.pdf",
                reference: str | None = None) -> str:
    """Two panels: error vs iteration and error vs cumulative wall time (baselines.py plot(time))."""
    plt = _plt()
    fig, axes = plt.subplots(1, 2, figsize=(13, 4.5))
    runs = [("Biscotti", trace, "red", "--")]
    if fedsys_trace:
        runs.append(("Federated Learning", fedsys_trace, "black", "-"))
    for label, path, color, ls in runs:
        rows = read_trace(path)
        it = [r["iteration"] for r in rows]
        err = [r["test_error"] for r in rows]
        t, acc = [], 0.0
        for r in rows:
            acc += r.get("wall_s", 0.0)
            t.append(acc)
        axes[0].plot(it, err, color=color, ls=ls, lw=2, label=label)
        axes[1].plot(t, err, color=color, ls=ls, lw=2, label=label)
    ref = _reference_series(reference, "mnist_poison_30_100.pdf", "No Poison")
    if ref:
        axes[0].plot(ref["x"], ref["y"], color="gray", ls=":", lw=1.5, label="reference FedSys (real MNIST)")
    _style(axes[0], "Training Iterations", "Test Error")
    _style(axes[1], "Time (s)", "Test Error")
    fig.tight_layout()
    fig.savefig(out)
    return out


def poisoning(trace: str, out: str = "eval_poisoning.pdf", reference: str | None = None,
              fedsys_trace: str | None = None) -> str:
    plt = _plt()
    fig, axes = plt.subplots(1, 2, figsize=(13, 4.5))
    for label, path, color, ls in [("Biscotti", trace, "red", "--")] + (
            [("Federated Learning", fedsys_trace, "black", "-")] if fedsys_trace else []):
        rows = read_trace(path)
        it = [r["iteration"] for r in rows]
        axes[0].plot(it, [r["test_error"] for r in rows], color=color, ls=ls, lw=2, label=label)
        axes[1].plot(it, [r.get("attack_rate", float("nan")) for r in rows], color=color, ls=ls, lw=2, label=label)
    for ax, pdf, lab in ((axes[0], "mnist_poison_30_100.pdf", "Biscotti"),
                         (axes[1], "mnist_poison_30_100_AR.pdf", "Biscotti")):
        ref = _reference_series(reference, pdf, lab)
        if ref:
            ax.plot(ref["x"], ref["y"], color="gray", ls=":", lw=1.5, label="reference Biscotti 30% (real MNIST)")
    _style(axes[0], "Training Iterations", "Test Error")
    _style(axes[1], "Training Iterations", "1-7 Attack Rate")
    fig.tight_layout()
    fig.savefig(out)
    return out


def breakdown(trace: str, out: str = "eval_cost_breakdown.pdf", skip: int = 5) -> str:
    """Mean per-phase host time per round (t_* fields of the trace), one stacked bar."""
    plt = _plt()
    rows = read_trace(trace)[skip:]
    keys = sorted({k for r in rows for k in r if k.startswith("t_") and "." not in k})
    means = {k[2:]: 1e3 * sum(r.get(k, 0.0) for r in rows) / max(1, len(rows)) for k in keys}
    fig, ax = plt.subplots(figsize=(6, 5))
    bottom = 0.0
    for name, v in sorted(means.items(), key=lambda kv: -kv[1]):
        ax.bar(["round"], [v], bottom=bottom, label=f"{name} ({v:.2f} ms)")
        bottom += v
    ax.set_ylabel("ms per round (host phases)", fontsize=14)
    ax.legend(fontsize=9, loc="upper left", bbox_to_anchor=(1.0, 1.0))
    fig.tight_layout()
    fig.savefig(out)
    return out


def scaling(bench_files: list[str], x: str = "peers", out: str = "eval_scaling.pdf") -> str:
    """s/round vs peers (increments) or vs GPUs (n_gpus) from bench.py result lines."""
    plt = _plt()
    pts = []
    for f in bench_files:
        b = read_bench(f)
        xv = b["config"].get("peers") if x == "peers" else b.get("n_gpus")
        pts.append((xv, 1e3 * b["value"]))
    pts.sort()
    fig, ax = plt.subplots(figsize=(6, 4.5))
    ax.plot([p[0] for p in pts], [p[1] for p in pts], "o-", color="red", lw=2, label="Biscotti on MI355X")
    _style(ax, "Peers" if x == "peers" else "GPUs", "ms per round", ylim=None)
    fig.tight_layout()
    fig.savefig(out)
    return out


def heatmap(bench_jsonl: list[str], out: str = "eval_poison_nsamples.pdf", metric: str = "attack_rate_last10_mean",
            rows: str = "poisoning", cols: str = "ns_percent") -> str:
    """Attack rate (or any bench metric) over poisoner fraction x % of updates collected, from bench
    result lines (eval/eval_poison_nsamples/plotHeatMap.py: 10-50 % poisoners x -ns 20/40/70)."""
    import numpy as np

    plt = _plt()
    cells = {}
    for f in bench_jsonl:
        with open(f) as fh:
            for ln in fh:
                if ln.startswith("{"):
                    b = json.loads(ln)
                    c = b.get("config")
                    if isinstance(c, dict) and metric in b and rows in c and cols in c:
                        cells[(c[rows], c[cols])] = b[metric]
    rv = sorted({k[0] for k in cells}, reverse=True)
    cv = sorted({k[1] for k in cells})
    grid = np.full((len(rv), len(cv)), np.nan)
    for (r, c), v in cells.items():
        grid[rv.index(r), cv.index(c)] = v
    fig, ax = plt.subplots(figsize=(7, 4.5))
    im = ax.imshow(grid, cmap="Greys", aspect="auto")
    for i in range(len(rv)):
        for j in range(len(cv)):
            if not np.isnan(grid[i, j]):
                ax.text(j, i, f"{grid[i, j]:.2f}", ha="center", va="center",
                        color="white" if grid[i, j] > 0.5 * np.nanmax(grid) else "black", fontsize=12)
    ax.set_xticks(range(len(cv)), [f"{c}%" for c in cv])
    ax.set_yticks(range(len(rv)), [f"{100 * r:.0f}%" for r in rv])
    ax.set_xlabel("Number (%) of received updates", fontsize=13)
    ax.set_ylabel("Percent of poisoners", fontsize=13)
    fig.colorbar(im, ax=ax, label=metric)
    fig.tight_layout()
    fig.savefig(out)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("convergence")
    c.add_argument("--trace", required=True)
    c.add_argument("--fedsys-trace")
    c.add_argument("--reference")
    c.add_argument("-o", "--out", default="eval_convrate.pdf")
    p = sub.add_parser("poisoning")
    p.add_argument("--trace", required=True)
    p.add_argument("--fedsys-trace")
    p.add_argument("--reference")
    p.add_argument("-o", "--out", default="eval_poisoning.pdf")
    b = sub.add_parser("breakdown")
    b.add_argument("--trace", required=True)
    b.add_argument("--skip", type=int, default=5)
    b.add_argument("-o", "--out", default="eval_cost_breakdown.pdf")
    s = sub.add_parser("scaling")
    s.add_argument("--bench", nargs="+", required=True)
    s.add_argument("--x", default="peers", choices=["peers", "gpus"])
    s.add_argument("-o", "--out", default="eval_scaling.pdf")
    h = sub.add_parser("heatmap")
    h.add_argument("--bench", nargs="+", required=True, help="bench JSON lines (files)")
    h.add_argument("--metric", default="attack_rate_last10_mean")
    h.add_argument("-o", "--out", default="eval_poison_nsamples.pdf")
    a = ap.parse_args(argv)
    if a.cmd == "convergence":
        print(convergence(a.trace, a.fedsys_trace, a.out, a.reference))
    elif a.cmd == "poisoning":
        print(poisoning(a.trace, a.out, a.reference, a.fedsys_trace))
    elif a.cmd == "breakdown":
        print(breakdown(a.trace, a.out, a.skip))
    elif a.cmd == "heatmap":
        print(heatmap(a.bench, a.out, a.metric))
    else:
        print(scaling(a.bench, a.x, a.out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
