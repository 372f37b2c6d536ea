"""Typed run configuration accepting the reference's flag names (DistSys/main.go:613-647)."""
from __future__ import annotations

import argparse
from dataclasses import dataclass, field, fields
from typing import ClassVar


@dataclass
class RunConfig:
    # --- reference flags
    num_nodes: int = 100            # -t
    node_index: int = -1            # -i  (per-process mode; SPMD runs host several peers per rank)
    dataset: str = "mnist"          # -d  mnist | creditcard
    peers_file: str | None = None   # -f
    my_ip: str = ""                 # -a
    my_private_ip: str = ""         # -pa
    port: str = ""                  # -p
    colluders: int = 0              # -c  percent
    num_miners: int = 3             # -na
    num_verifiers: int = 3          # -nv
    num_noisers: int = 2            # -nn
    secure_agg: bool = True         # -sa
    noising: bool = True            # -np
    verification: bool = True       # -vp
    epsilon: float = 2.0            # -ep
    poisoning: float = 0.0          # -po
    perc_samples: int = 70          # -ns
    rand_sample: bool = False       # -rs
    # --- compile-time constants of the reference (main.go:28-58, honest.go:44-57)
    defense: str = "KRUM"           # POISON_DEFENSE (KRUM | RONI), or LSH (the sieve of ML/code/logistic_aggregator.py)
    max_iterations: int = 100       # MAX_ITERATIONS
    poly_size: int = 10             # POLY_SIZE
    precision: int = 4              # PRECISION
    batch_size: int = 10
    default_stake: int = 10
    stake_unit: int = 5
    # --- framework knobs
    seed: int = 0
    churn: float = 0.0              # fraction of peers offline per round (fault-tolerance runs)
    churn_kill_per_min: float = 0.0  # process churn (eval/eval_FT): peers killed per minute, restarted after
    #                                  60/rate - 5 s with fresh VRF keys, rejoining through chain sync
    partition: str = ""             # network partition injection (DistSys/blockNode.sh drops one peer's port
    #                                 for 30 s): "peer:first_iteration:rounds[,...]" -- the peer is
    #                                 unreachable (and unreaching) for those rounds
    fail_at: str = ""               # fault injection "IT[@RANK]": that rank (default 0) dies right after
    #                                 committing iteration IT (the reference's FAIL_PROB crash, made
    #                                 deterministic; torchrun restarts the job from chain_file)
    data_dir: str | None = None     # real MNIST .npy shards (reference layout), else synthetic
    commit_key: str | None = None   # commitKey.json (else generated: PK[i] = 2^i G1, s = 2)
    pkey_file: str | None = None    # pKeyG1.json (else derived from seed)
    verify_signatures: bool = False  # miners check verifier signatures (commented out in reference, Q5)
    host_threads: int = 16          # native crypto pool of this rank (bench.py sizes it from the CPU quota)
    lazy_eval: bool = False         # GPU: a round's test error / attack rate are read (and logged) in the next
    #                                 round's VRF wait or by drain(), not at its end (bench.py sets it)
    log_dir: str | None = None
    trace_file: str | None = None
    chain_file: str | None = None   # append-only chain persistence (checkpoint / resume)
    resume: bool = False
    device: str | None = None       # "cpu" forces the CPU path
    log_every_peer: bool = False    # one Train Error line per local peer (reference style)
    phase_log: bool = False         # the reference's role / phase lines (Verifiers are, Getting noise from, Sending
    #                                 update to verifiers / miners, Got share for, Sending block of iteration) so its
    #                                 parseLogs.py phase breakdown works on our logs (protocol/golog.py)
    deterministic_time: bool = False  # block timestamps = iteration + 1 (reproducible chains in tests)
    miner_threshold: str = "half_samples"  # when the leader miner builds its block from the shares it has
    #                                 (secure path; its block holds the first arrivals up to that count):
    #   half_samples  NUM_SAMPLES/2 shares (main.go:360, the reference's live rule; default)
    #   eighth        numberOfNodes/8, at least 2 (minBlockSize, main.go:348-352: the commented-out rule)
    #   tenth         numberOfNodes/10, at least 2: what the nsdi-eval/churn logs fired at ("As miner, I expect
    #                 5 shares" with 50 peers, 60s.log:9686; an older main.go whose log lines are at :304-314)
    #                 The plain path's leader keeps NUM_SAMPLES/2 updates (processUpdate, main.go:1222-1230).
    phase_sync: bool = False        # device sync at phase boundaries (diagnostics: per-phase GPU times)
    audit_aggregate: bool = True    # check the recovered aggregate against the miners' summed chunk
    #                                 commitments (verifyCommitment on the aggregate; not in the reference)
    comm_timeout_s: float = 300.0   # collective timeout: a dead rank fails the job instead of hanging it
    vrf_device: bool = True         # GPU: the VRF proofs nothing reads (roles proof Q7, the noiser proofs)
    #                                 run on the device (kernels/vrf.hip); the host computes only the
    #                                 64-byte outputs the lottery consumes
    kzg_audit: str = "off"          # batched verifySecret (kyber.go:650-673) over every (chunk, share point) of
    #                                 the aggregate: off | consistent (y against PK[poly*k]) | literal (y
    #                                 against G1: the reference's formula, which only chunk 0 satisfies, Q9).
    #                                 Device RLC sums (kzg.hip) + one host 3-pairing product per batch of
    #                                 rounds, joined lazily; failures are counted and logged, never block the chain
    ablation: str = ""              # comma list of semantic / pipeline ablations (experiments and tests only):
    #   noise_independent  each worker draws private noise instead of its noisers' shared pre-sampled
    #                      vectors (client_obj.py:97-98 shares them; docs/ROBUSTNESS.md)
    #   shared_inbox       all verifiers judge one inbox (round-1 model; the reference: krum.go:284-322)
    #   no_miner_cap       the leader's block takes every approved update, not its first NUM_SAMPLES/2
    #   no_roles_proof     skip the discarded getVRFRoles proof (Q7)
    #   no_pipeline        GPU: no cross-round pipelining (pre-step, pre-Gram, early VRF, next-round MSM
    #                      at block build): the chain must not change (tests)
    #   spec_head_shared   GPU: the next round's share MSM at block build also when several ranks share one
    #                      GPU (off there by default: rehearsals of the one-rank-per-GPU path force it)
    #   spec_all_candidates GPU: the speculative share MSM covers every candidate (every approved worker's
    #                      shares, as each reference worker computes its own), not only the leader's first
    #                      arrivals up to the adaptive horizon (head.py SPEC_MARGIN): the chain must not change
    #   short_spin         GPU: host waits spin 200 us before polling with sleeps also with one rank (the
    #                      multi-rank setting; one rank spins up to 5 ms: a sleeping thread wakes late)
    #   noise_gram_each_round GPU: the noise-aware Gram computes its noise x noise tiles every round instead of
    #                      copying them from the setup table of the 100 periodic noise Grams (ml.NoiseRows.gram_table)
    #   no_early_front     GPU: the next round's noiser lottery + Krum launch run at its own start instead of at
    #                      the end of the previous round (engine._round_front): the chain must not change
    #   spec_tight         GPU: the speculative MSM's horizon is the leader's cap exactly (no margin, no slack): a
    #                      block reaching past its first cap arrivals is a speculative miss, topped up by the host
    #                      path (tests and measurements of that path): the chain must not change
    #   wave_prio_multi    GPU: the round kernels' wave priority classes (kernels/wave_prio.h) also with several
    #                      ranks (default: one rank only; the collectives' kernels run at the default class)
    #   multi_early_front  GPU, several ranks with the native collectives: the next round's front at the end of the
    #                      previous round as with one rank (engine._early_front_ok; measured slower there)
    #   side_prio_low      GPU: the full-commitment sums (k_segment_sum) and the aggregate audit (k_chunk_check) one
    #                      wave-priority class below the speculative share MSM instead of at the critical class
    #   witness_sums_tree  GPU: the miners' witness sums in k_sum_rows2's LDS-tree form (16 lanes a column) instead of
    #                      one lane a column (k_sum_cols_serial: ~30 % fewer Jacobian additions)
    #   side_all_cus       GPU: the speculative share MSM's stream on every CU (default: 3/4 of them, the rest kept for
    #                      the critical path)
    #   no_spec_front      GPU, one rank: the next round's front at the commit of the block (after the audit wait and
    #                      the read-back) instead of right after the block's build (engine._spec_front_launch): the
    #                      chain must not change
    #   multi_spec_front   GPU, several ranks with the native collectives: the speculative front as with one rank
    #                      (engine._spec_front_ok; measured slower there)

    # seconds per reference round: maps the churn scripts' seconds onto rounds (the reference's churn runs
    # took 25-31 s per round, nsdi-eval/churn/*.log)
    churn_round_s: ClassVar[float] = 25.44
    MINER_THRESHOLDS: ClassVar[dict] = {"half_samples": 0, "eighth": 8, "tenth": 10}   # -> miner_block_div
    ABLATIONS: ClassVar[tuple] = ("noise_independent", "shared_inbox", "no_miner_cap", "no_roles_proof", "no_pipeline",
                                  "spec_head_shared", "spec_all_candidates", "short_spin",
                                  "noise_gram_each_round", "spec_tight", "no_early_front",
                                  "wave_prio_multi", "multi_early_front", "side_prio_low",
                                  "witness_sums_tree", "side_all_cus", "no_spec_front",
                                  "multi_spec_front")

    def has(self, ablation: str) -> bool:
        """True when `ablation` (one of ABLATIONS) is switched on."""
        assert ablation in self.ABLATIONS, ablation
        got = self.__dict__.get("_ablation_set")   # the round asks ~11 times: parsed once per ablation string
        if got is None or got[0] != self.ablation:
            got = self.__dict__["_ablation_set"] = (self.ablation, frozenset(a.strip() for a in self.ablation.split(",")))
        return ablation in got[1]

    @property
    def noise_independent(self) -> bool:
        return self.has("noise_independent")

    @property
    def roles_vrf_proof(self) -> bool:
        return not self.has("no_roles_proof")

    def fail_point(self) -> tuple[int, int]:
        """(iteration, rank) of the injected crash; iteration -1 when none."""
        if not self.fail_at:
            return -1, 0
        it, _, rank = str(self.fail_at).partition("@")
        return int(it), int(rank or 0)

    def validate(self) -> None:
        """Reject configurations the kernels cannot run, up front (instead of a launch error in the
        middle of a round).  Limits: committee Multi-Krum <= 8192 candidate rows, inbox <= 4096,
        <= 64 verifiers (ml.hip KC1-KC3); exact recovery <= 32 share points per chunk and poly <= 16
        (k_recover_w); local step B <= 16 and <= 16 classes (k_softmax_step); <= 16 noisers."""
        import math

        err = []
        if self.dataset not in ("mnist", "lfw", "creditcard"):
            err.append(f"dataset {self.dataset!r}: expected mnist | lfw | creditcard")
        if self.num_nodes < 2:
            err.append("need at least 2 nodes")
        committee = self.num_verifiers + self.num_miners
        if self.num_nodes - committee < 1:
            err.append(f"{self.num_nodes} nodes leave no worker beside {committee} committee members")
        workers = max(0, self.num_nodes - min(committee, self.num_nodes))
        if workers > 8192:
            err.append(f"{workers} workers per round: committee Krum takes at most 8192 candidates")
        thresh = min(int(self.num_nodes * self.perc_samples / 100.0), max(workers, 0))
        if self.rand_sample:
            thresh = max(workers, 0)
        if self.verification and thresh > 4096:
            err.append(f"verifier inbox of {thresh} updates: committee Krum takes at most 4096 per verifier")
        if self.num_verifiers > 64:
            err.append("at most 64 verifiers")
        if self.num_miners <= 0 or self.num_verifiers < 0 or self.num_noisers < 0:
            err.append("committee sizes must be non-negative (and >= 1 miner)")
        elif math.ceil(2 * self.poly_size / self.num_miners) * self.num_miners > 32:
            err.append("TOTAL_SHARES = ceil(2 POLY_SIZE / miners) * miners must be <= 32")
        if not 2 <= self.poly_size <= 16:
            err.append("POLY_SIZE must be in 2..16")
        if self.dataset in ("mnist", "lfw") and not 1 <= self.batch_size <= 16:
            err.append("softmax local step: batch size 1..16")
        if self.num_noisers > 16 or (self.noising and self.num_noisers >= self.num_nodes):
            err.append("noisers: at most 16 and fewer than the nodes")
        if not 0.0 <= self.poisoning < 1.0 or not 0.0 <= self.churn < 1.0:
            err.append("poisoning / churn fractions must be in [0, 1)")
        try:
            for peer, first, rounds in self.partitions():
                if not (0 <= peer < self.num_nodes) or rounds < 1:
                    err.append(f"partition {peer}:{first}:{rounds}: peer out of range or no rounds")
        except ValueError:
            err.append(f"partition {self.partition!r}: expected peer:first_iteration:rounds[,...]")
        bad = {a.strip() for a in self.ablation.split(",") if a.strip()} - set(self.ABLATIONS)
        if bad:
            err.append(f"unknown ablation(s) {sorted(bad)}: expected {', '.join(self.ABLATIONS)}")
        try:
            self.fail_point()
        except ValueError:
            err.append(f"fail_at {self.fail_at!r}: expected IT or IT@RANK")
        if self.defense not in ("KRUM", "RONI", "LSH"):
            err.append(f"defense {self.defense!r}: expected KRUM | RONI | LSH")
        if self.miner_threshold not in self.MINER_THRESHOLDS:
            err.append(f"miner_threshold {self.miner_threshold!r}: expected {' | '.join(self.MINER_THRESHOLDS)}")
        if self.kzg_audit not in ("off", "consistent", "literal"):
            err.append(f"kzg_audit {self.kzg_audit!r}: expected off | consistent | literal")
        if err:
            raise ValueError("invalid RunConfig: " + "; ".join(err))

    def partitions(self) -> list[tuple[int, int, int]]:
        """The partition schedule as (peer, first iteration, rounds) triples."""
        out = []
        for item in filter(None, (x.strip() for x in self.partition.split(","))):
            peer, first, rounds = (int(v) for v in item.split(":"))
            out.append((peer, first, rounds))
        return out

    def protocol(self, rt):
        pc = rt.ProtocolConfig()
        pc.num_nodes = self.num_nodes
        pc.num_verifiers = self.num_verifiers
        pc.num_miners = self.num_miners
        pc.num_noisers = self.num_noisers
        pc.secure_agg = self.secure_agg
        pc.noising = self.noising
        pc.verification = self.verification
        pc.epsilon = self.epsilon
        pc.poisoning = self.poisoning
        pc.perc_samples = self.perc_samples
        pc.rand_sample = self.rand_sample
        pc.colluders = self.colluders
        pc.defense = self.defense
        pc.poly_size = self.poly_size
        pc.precision = self.precision
        pc.max_iterations = self.max_iterations
        pc.default_stake = self.default_stake
        pc.stake_unit = self.stake_unit
        pc.seed = self.seed & (2**64 - 1)
        pc.shared_inbox = self.has("shared_inbox")
        pc.miner_cap = not self.has("no_miner_cap")
        pc.miner_block_div = self.MINER_THRESHOLDS.get(self.miner_threshold, 0) if self.secure_agg else 0
        pc.derive()
        return pc


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "t", "yes", "y")


def add_reference_flags(ap: argparse.ArgumentParser) -> None:
    """Register the DistSys flags (single-dash, Go style) on an argparse parser."""
    ap.add_argument("-t", dest="num_nodes", type=int, default=100, help="total number of nodes")
    ap.add_argument("-i", dest="node_index", type=int, default=-1, help="this node's index")
    ap.add_argument("-d", dest="dataset", default="mnist", help="dataset (mnist | creditcard)")
    ap.add_argument("-f", dest="peers_file", default=None, help="peers file (IP:port per line)")
    ap.add_argument("-a", dest="my_ip", default="", help="public IP")
    ap.add_argument("-pa", dest="my_private_ip", default="", help="private IP")
    ap.add_argument("-p", dest="port", default="", help="port")
    ap.add_argument("-c", dest="colluders", type=int, default=0, help="colluders (percent)")
    ap.add_argument("-na", dest="num_miners", type=int, default=3, help="number of aggregators")
    ap.add_argument("-nv", dest="num_verifiers", type=int, default=3, help="number of verifiers")
    ap.add_argument("-nn", dest="num_noisers", type=int, default=2, help="number of noisers")
    ap.add_argument("-sa", dest="secure_agg", type=_bool, default=True, help="secure aggregation on/off")
    ap.add_argument("-np", dest="noising", type=_bool, default=True, help="noising on/off")
    ap.add_argument("-vp", dest="verification", type=_bool, default=True, help="verification on/off")
    ap.add_argument("-ep", dest="epsilon", type=float, default=2.0, help="epsilon")
    ap.add_argument("-po", dest="poisoning", type=float, default=0.0, help="poisoner fraction")
    ap.add_argument("-ns", dest="perc_samples", type=int, default=70, help="percent of updates collected")
    ap.add_argument("-rs", dest="rand_sample", type=_bool, default=False, help="random sampling")


def add_framework_flags(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--defense", default="KRUM", choices=["KRUM", "RONI", "LSH"])
    ap.add_argument("--max-iterations", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--churn", type=float, default=0.0)
    ap.add_argument("--churn-kill-per-min", type=float, default=0.0)
    ap.add_argument("--partition", default="", help="peer:first_iteration:rounds[,...] unreachable (blockNode.sh)")
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--commit-key", default=None)
    ap.add_argument("--pkey-file", default=None)
    ap.add_argument("--no-roles-vrf-proof", dest="no_roles_vrf_proof", action="store_true",
                    help="skip the discarded getVRFRoles proof (ablation no_roles_proof)")
    ap.add_argument("--ablation", default="", help="comma list of RunConfig.ABLATIONS (experiments)")
    ap.add_argument("--verify-signatures", action="store_true")
    ap.add_argument("--host-threads", type=int, default=16)
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--trace-file", default=None)
    ap.add_argument("--chain-file", default=None)
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--device", default=None)
    ap.add_argument("--log-every-peer", action="store_true")
    ap.add_argument("--phase-log", action="store_true",
                    help="write the reference's role and phase log lines (parseLogs.py breakdowns)")
    ap.add_argument("--deterministic-time", action="store_true")
    ap.add_argument("--miner-threshold", default="half_samples", choices=sorted(RunConfig.MINER_THRESHOLDS),
                    help="shares the leader miner builds its block at: NUM_SAMPLES/2 (main.go:360), N/8 "
                         "(main.go:348-352) or N/10 (the nsdi-eval/churn logs)")
    ap.add_argument("--phase-sync", action="store_true",
                    help="synchronise the device at every phase boundary (per-phase GPU times; slower)")
    ap.add_argument("--no-audit-aggregate", dest="audit_aggregate", action="store_false")
    ap.add_argument("--no-vrf-device", dest="vrf_device", action="store_false",
                    help="compute every VRF proof on host threads")
    ap.add_argument("--kzg-audit", default="off", choices=["off", "consistent", "literal"],
                    help="batched verifySecret over each round's aggregate (K13)")
    ap.add_argument("--comm-timeout", dest="comm_timeout_s", type=float, default=300.0)
    ap.add_argument("--fail-at", type=int, default=-1, help="fault injection: die after committing this iteration")
    ap.add_argument("--fail-rank", type=int, default=0, help="the rank --fail-at kills")


def config_from_args(ns: argparse.Namespace) -> RunConfig:
    """RunConfig from parsed reference + framework flags (flags the config has no field for, such as a
    CLI's own --rounds, are ignored)."""
    names = {f.name for f in fields(RunConfig)}
    v = vars(ns)
    kw = {k: x for k, x in v.items() if k in names}
    abl = [a for a in str(v.get("ablation", "") or "").split(",") if a.strip()]
    if v.get("no_roles_vrf_proof"):
        abl.append("no_roles_proof")
    kw["ablation"] = ",".join(dict.fromkeys(a.strip() for a in abl))
    if int(v.get("fail_at", -1) if v.get("fail_at") is not None else -1) >= 0:
        kw["fail_at"] = f"{int(v['fail_at'])}@{int(v.get('fail_rank', 0) or 0)}"
    else:
        kw.pop("fail_at", None)
    return RunConfig(**kw)
