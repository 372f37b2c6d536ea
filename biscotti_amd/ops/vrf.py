"""Device ECVRF prover (kernels/vrf.hip): RFC 9381 ECVRF-EDWARDS25519-SHA512-TAI proofs on gfx950.

The protocol computes two VRF proofs per peer per round that nothing reads (the roles proof of
getVRFRoles, quirk Q7, and the proof half of every worker's noiser VRF, vrf.go:54-100 -- only the
64-byte output feeds the lottery).  Round 1 spent ~37 ms of host CPU per round on them; here the
host computes the outputs the lottery needs (VrfJob outputs_only) and the proofs are queued for the
device, batch_rounds rounds per launch on a low-priority stream; the kernel splits each proof over the
three waves of a workgroup, so a launch's latency is about one variable-base scalar multiplication.  Bit-exact with runtime/vrf.cpp
(tests/test_gpu_vrf.py), which is itself pinned to the RFC's example vector.
"""
from __future__ import annotations

import numpy as np
import torch

from ..native import hip, rt
from ..utils import h2d
from ..utils import streams as S

_TORCH_OF = {np.dtype(np.int32): torch.int32, np.dtype(np.uint8): torch.uint8}


def _i32(b: bytes) -> np.ndarray:
    return np.frombuffer(b, np.uint8).view(np.int32)


class DeviceVrfProver:
    ALPHA_LEN = 32

    def __init__(self, device, batch_rounds: int = 1):
        self.device = torch.device(device)
        self.btab = torch.from_numpy(_i32(rt().vrf_base_table()).copy()).to(self.device)   # [512 * 32]
        self.batch_rounds = max(1, int(batch_rounds))
        self._bufs: dict = {}
        self._row: dict[bytes, int] = {}
        self._keys: list[np.ndarray] = []
        self._keys_dev = None
        self._queue: list[tuple[list[int], bytes]] = []
        self._inflight: list = []
        self.proofs = 0

    def _rows(self, seeds) -> list[int]:
        out = []
        for s in seeds:
            r = self._row.get(s)
            if r is None:
                r = self._row[s] = len(self._keys)
                self._keys.append(_i32(rt().vrf_key_material(s)))
                self._keys_dev = None
            out.append(r)
        return out

    def prove(self, seeds, alphas, beta: bool = False):
        """Proofs of seeds[i] over alphas[i] (32-byte messages) on the current stream: (pi uint8
        [n, 80], beta uint8 [n, 64] or None).  Asynchronous: read the tensors after a sync."""
        assert len(alphas) == len(seeds) and all(len(a) == self.ALPHA_LEN for a in alphas)
        uniq = {a: i for i, a in enumerate(dict.fromkeys(alphas))}
        return self._launch(np.asarray(self._rows(seeds), np.int32), list(uniq),
                            np.asarray([uniq[a] for a in alphas], np.int32), beta)

    def _launch(self, rows: np.ndarray, alphas: list, alpha_idx: np.ndarray, beta: bool = False, reuse: bool = False,
                urgent: bool = False):
        n = int(rows.size)
        if self._keys_dev is None:
            self._keys_dev = self._upload(np.concatenate(self._keys))
        al = self._upload(np.frombuffer(b"".join(alphas), np.uint8))
        idx = self._upload(np.concatenate([rows, alpha_idx]))
        # scratch and the (discarded) proofs reuse one buffer per stream: launches on a stream run in order,
        # and a fresh multi-MB allocation inside a timed round could cost a hipMalloc
        key = S.raw()
        buf = self._bufs.get(key) if reuse else None
        if not reuse:
            buf = (torch.empty((max(n, 1), 320), dtype=torch.int32, device=self.device),
                   torch.empty((max(n, 1), 80), dtype=torch.uint8, device=self.device))
        elif buf is None or buf[0].shape[0] < max(n, 1):
            cap = max(n, 1, self.batch_rounds * 256)
            buf = self._bufs[key] = (torch.empty((cap, 320), dtype=torch.int32, device=self.device),
                                     torch.empty((cap, 80), dtype=torch.uint8, device=self.device))
        scratch, pi = buf[0][: max(n, 1)], buf[1][:n]
        bt = torch.empty((n, 64), dtype=torch.uint8, device=self.device) if beta else None
        err = hip().bsc_vrf_prove_p(self._keys_dev.data_ptr(), idx.data_ptr(), al.data_ptr(), idx[n:].data_ptr(),
                                    self.ALPHA_LEN, n, self.btab.data_ptr(), scratch.data_ptr(), pi.data_ptr(),
                                    bt.data_ptr() if bt is not None else None, int(urgent), S.raw())
        if err != 0:
            raise RuntimeError(f"HIP launch of vrf_prove failed with hipError {err}")
        self.proofs += n
        return pi, bt

    def reserve(self, stream, n: int) -> None:
        """Allocate the batched launches' scratch / proof buffers for n proofs now (engine warm-up), not at
        the first flush inside the timed rounds."""
        with S.use(stream):
            key = S.raw()
            cap = max(n, 1, self.batch_rounds * 256)
            buf = self._bufs.get(key)
            if buf is None or buf[0].shape[0] < cap:
                self._bufs[key] = (torch.empty((cap, 320), dtype=torch.int32, device=self.device),
                                   torch.empty((cap, 80), dtype=torch.uint8, device=self.device))

    def _upload(self, a: np.ndarray) -> torch.Tensor:
        # through the pinned staging ring (utils.h2d), stream-ordered: a pageable .to(device) blocks
        # behind the round's queued kernels, and a fresh pin_memory() costs ~1 ms of host time
        return h2d(np.ascontiguousarray(a), _TORCH_OF[a.dtype], self.device)

    # ---- round-batched queue: the engine submits each round's proofs, one launch per batch_rounds
    def submit(self, seeds, alpha: bytes, stream) -> None:
        """seeds: the proving keys' seeds, or already their key rows (int32 array, _rows)."""
        if len(seeds):
            # key rows resolved now, so a flush only concatenates
            rows = seeds if isinstance(seeds, np.ndarray) else np.asarray(self._rows(seeds), np.int32)
            self._queue.append((rows, bytes(alpha)))
        if len(self._queue) >= self.batch_rounds:
            self.flush(stream)

    def flush(self, stream, urgent: bool = False) -> None:
        """Launch the queued rounds' proofs.  urgent: the caller's next step waits for them (the run's final
        flush) -- they run at the highest wave priority instead of filling the round's idle issue slots."""
        if not self._queue:
            return
        q, self._queue = self._queue, []
        if len(q) == 1:
            # one round (one message): rows, zero message indices and the 32-byte message in ONE upload
            rows, alpha = q[0]
            n = int(rows.size)
            buf = np.zeros(2 * n + len(alpha) // 4, np.int32)
            buf[:n] = rows
            buf[2 * n:] = np.frombuffer(alpha, np.int32)
            with S.use(stream):
                if self._keys_dev is None:
                    self._keys_dev = self._upload(np.concatenate(self._keys))
                up = self._upload(buf)
                scratch = torch.empty((n, 320), dtype=torch.int32, device=self.device)
                pi = torch.empty((n, 80), dtype=torch.uint8, device=self.device)
                err = hip().bsc_vrf_prove_p(self._keys_dev.data_ptr(), up.data_ptr(), up[2 * n:].data_ptr(),
                                            up[n:].data_ptr(), self.ALPHA_LEN, n, self.btab.data_ptr(),
                                            scratch.data_ptr(), pi.data_ptr(), None, int(urgent), S.raw())
                if err != 0:
                    raise RuntimeError(f"HIP launch of vrf_prove failed with hipError {err}")
                self.proofs += n
                ev = S.record(stream)
            self._inflight.append((ev, (pi, scratch, up)))
            self._inflight = [x for x in self._inflight if not x[0].query()] if len(self._inflight) > 4 \
                else self._inflight
            return
        rows = np.concatenate([r for r, _ in q])
        alpha_idx = np.repeat(np.arange(len(q), dtype=np.int32), [r.size for r, _ in q])
        with S.use(stream):   # uploads, scratch and the launch all on the prover's stream
            pi, _ = self._launch(rows, [a for _, a in q], alpha_idx, reuse=True, urgent=urgent)
            ev = S.record(stream)
        self._inflight.append((ev, pi))
        # keep the last few batches alive until their kernels finished (the proofs are discarded)
        self._inflight = [x for x in self._inflight if not x[0].query()] if len(self._inflight) > 2 else self._inflight

    def drain(self, stream) -> None:
        self.flush(stream, urgent=True)
        for ev, _ in self._inflight:
            S.host_wait(ev)
        self._inflight = []
