"""Analytical committee-security models of the reference's eval (eval/eval_vrf_security/vrf_security.py,
eval/eval_privacy_noise_attack/vrf_noise_security.py), plus an empirical check against this
framework's own stake lottery.

* Committee capture: an adversary holding a fraction s of the stake takes a strict majority of a
  c-member committee with probability sum_{i > c/2} C(c, i) s^i (1 - s)^(c - i) when members are
  drawn by stake with replacement (the reference's binomial model).  The lottery here draws c
  *distinct* peers (RoundFSM / Lottery); with K of N equal-stake peers adversarial that is the
  hypergeometric tail sum_{i > c/2} C(K, i) C(N - K, c - i) / C(N, c).
* Noise unmasking (the privacy attack of eval_privacy_noise_attack): a worker's DP noise is known to
  the adversary when all nn of its noisers collude; the attack needs the noised update, seen by the
  verifiers.  The reference multiplies s^nn by (1 - s^nv) (`vrf_noise_security.py`, kept as
  `noise_attack_prob_reference`); the event "all noisers and at least one verifier adversarial" is
  s^nn (1 - (1 - s)^nv) (`noise_attack_prob`).

    python -m biscotti_amd.utils.vrf_security committee --peers 100 -o committee.pdf
    python -m biscotti_amd.utils.vrf_security noise -o noise.pdf
"""
from __future__ import annotations

import argparse
import sys
from math import comb


def majority_capture_prob(committee: int, stake: float) -> float:
    """P(strict adversarial majority) for c members drawn by stake with replacement."""
    return sum(comb(committee, i) * stake ** i * (1 - stake) ** (committee - i)
               for i in range(committee // 2 + 1, committee + 1))


def majority_capture_prob_distinct(peers: int, adversarial: int, committee: int) -> float:
    """P(strict adversarial majority) for c distinct members out of N equal-stake peers, K adversarial."""
    total = comb(peers, committee)
    return sum(comb(adversarial, i) * comb(peers - adversarial, committee - i)
               for i in range(committee // 2 + 1, min(committee, adversarial) + 1)) / total


def min_committee_size(stake: float, threshold: float, max_size: int = 200) -> int | None:
    """Smallest committee (>= 3) whose capture probability is below `threshold` (None: none up to max)."""
    for c in range(3, max_size + 1):
        if majority_capture_prob(c, stake) < threshold:
            return c
    return None


def noise_attack_prob(stake: float, noisers: int, verifiers: int) -> float:
    return stake ** noisers * (1 - (1 - stake) ** verifiers)


def noise_attack_prob_reference(stake: float, noisers: int, verifiers: int) -> float:
    return stake ** noisers * (1 - stake ** verifiers)


def simulate_verifier_capture(rt, peers: int, colluder_pct: int, verifiers: int, trials: int, seed0: int = 0) -> float:
    """Fraction of rounds in which the colluding peers (the top colluder_pct % of ids, as in the
    reference's collusion experiment) hold a strict majority of the verifiers, drawn by this
    framework's own stake lottery (`select_roles`, equal stake) over random block hashes."""
    import hashlib
    import math

    stake = {p: 10 for p in range(peers)}
    thresh = math.ceil(peers * (1 - colluder_pct / 100.0))
    hits = 0
    for t in range(trials):
        h = hashlib.sha256(f"round-{seed0}-{t}".encode()).digest()
        vs, _ = rt.select_roles(stake, h, verifiers, 1, peers)
        hits += sum(1 for v in vs if v >= thresh) > len(vs) // 2
    return hits / trials


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def plot_committee(out: str, stakes=(0.05, 0.1, 0.15, 0.2, 0.25, 0.3, 0.35),
                   thresholds=(0.001, 0.01, 0.05)) -> str:
    plt = _plt()
    fig, ax = plt.subplots(figsize=(8, 4.5))
    for th in thresholds:
        sizes = [min_committee_size(s, th) for s in stakes]
        ax.plot([100 * s for s in stakes], sizes, "o-", lw=2, label=f"P(capture) < {th}")
    ax.set_xlabel("adversarial stake (%)")
    ax.set_ylabel("committee size needed")
    ax.legend()
    fig.tight_layout()
    fig.savefig(out)
    return out


def plot_noise(out: str, stakes=tuple(x / 20 for x in range(1, 11)), noisers=(3, 5, 10), verifiers: int = 3) -> str:
    plt = _plt()
    fig, ax = plt.subplots(figsize=(8, 4.5))
    for nn in noisers:
        ax.plot([100 * s for s in stakes], [noise_attack_prob(s, nn, verifiers) for s in stakes], "o-", lw=2,
                label=f"# noisers = {nn}")
    ax.set_xlabel("adversarial stake (%)")
    ax.set_ylabel("P(noise unmasked)")
    ax.set_yscale("log")
    ax.legend()
    fig.tight_layout()
    fig.savefig(out)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("committee")
    c.add_argument("-o", "--out", default="vrf_committee_security.pdf")
    n = sub.add_parser("noise")
    n.add_argument("-o", "--out", default="vrf_noise_security.pdf")
    a = ap.parse_args(argv)
    print(plot_committee(a.out) if a.cmd == "committee" else plot_noise(a.out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
