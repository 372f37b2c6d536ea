"""The reference's phase and role log lines (RunConfig.phase_log, peer.py --phase-log).
Formats: DistSys/main.go:332,510-512,1405,1516,1550,1563,1692.  The lines are written after the
round from the phase timer's wall-clock stamps, so eval/eval_performance/parseLogs.py:92-185 can
rebuild the noise, verification and sec-agg times from them.  Each "where" tag is 11 characters
long, like main.go:NNN, because parseLogs.py slices "Miners are" lines at a fixed offset.
"""
from __future__ import annotations

from ..utils import fast_info_at

_W_ROLES, _W_NOISE, _W_VERIFY, _W_MINERS, _W_SHARE, _W_BLOCK = (
    "golog.py:10", "golog.py:20", "golog.py:30", "golog.py:40", "golog.py:50", "golog.py:60")


def _ids(xs) -> str:
    return "[" + " ".join(str(int(x)) for x in xs) + "]"   # Go's %v of []int


class GoPhaseLog:
    """Writes one round's reference lines for the logging peer `me` (the rank's first peer, whose Train
    Error lines the engine also writes).  The leader's two aggregation lines go into the same log.  On
    one rank with a log directory they also go into log_<leader>_<N>.log, the leader's own file, which
    is where parseLogs.py looks for them."""

    def __init__(self, log, me: int, num_nodes: int, addresses=None, log_dir: str | None = None,
                 world: int = 1):
        self.log, self.me, self.N = log, int(me), int(num_nodes)
        self.addrs = list(addresses) if addresses else [f"127.0.0.1:{8000 + i}" for i in range(self.N)]
        self.dir = log_dir if world == 1 else None
        self._files: dict = {}

    def _leader_line(self, leader: int, where: str, msg: str, when: float) -> None:
        fast_info_at(self.log, where, msg, when)
        if self.dir is None or leader == self.me:
            return
        from ..utils import get_logger

        lg = self._files.get(leader)
        if lg is None:
            lg = self._files[leader] = get_logger("peer", f"{self.dir}/log_{leader}_{self.N}.log")
        fast_info_at(lg, where, msg, when)

    def round(self, it: int, plan, stamps: dict, noisers: dict, approved, secure_agg: bool, noising: bool) -> None:
        """plan: the round's PlanView (verifiers, miners, workers, leader); stamps: phase -> (wall start,
        wall end); noisers: worker -> its noiser ids; approved: the workers with enough signatures."""
        me = self.me
        t0 = stamps.get("roles", (None, None))[0]
        if t0 is None:
            return
        nz = noisers.get(me, []) if noisers else []
        fast_info_at(self.log, _W_ROLES, f"Verifiers are {_ids(plan.verifiers)}", t0)
        fast_info_at(self.log, _W_ROLES, f"Miners are {_ids(plan.miners)}", t0)
        fast_info_at(self.log, _W_ROLES, f"Noisers are {_ids(nz)}", t0)
        ver = stamps.get("verify")
        if me in plan.workers and me not in plan.verifiers and me not in plan.miners and ver is not None:
            ns = stamps.get("noise")
            if noising and nz and ns is not None:
                addrs = "[" + " ".join(self.addrs[j] for j in nz) + "]"
                fast_info_at(self.log, _W_NOISE, f"{me}:Getting noise from {addrs}", ns[0])
            fast_info_at(self.log, _W_VERIFY, f"Sending update to verifiers. Iteration:{it}", ver[0])
            if me in set(approved):
                fast_info_at(self.log, _W_MINERS, "Sending update to miners", ver[1])
            else:
                fast_info_at(self.log, _W_MINERS, f"{me}:Couldn't get enough signatures. Iteration:{it}", ver[1])
        blk = stamps.get("block")
        if secure_agg and ver is not None and blk is not None:
            ld = int(plan.leader)
            self._leader_line(ld, _W_SHARE, f"{ld}:Got share for {it}, I am at {it}", ver[1])
            self._leader_line(ld, _W_BLOCK, f"{ld}:Sending block of iteration: {it}", blk[1])

    def flush(self) -> None:
        from ..utils import flush_logs

        for lg in self._files.values():
            flush_logs(lg)
