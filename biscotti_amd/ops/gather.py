"""The verification all_gather of several ranks as resident buffers and two kernels (kernels/gather.hip).

Per round, every rank sends ONE row [split Gram slot | its peers' commitment rows | noiser ids | noiser weights]
and receives every rank's; the row is gathered in place in a resident [world, row_bytes] buffer (two of them,
alternating by iteration: the Gram kernel of the next round writes its slot while this round's is still being
read).  The Gram slot is written by the Gram kernel itself (gram_stacked_async(out=...)), the rest by ONE pack
kernel with the noiser ids / weights in its arguments; ONE unpack kernel then produces the tiled Gram, the flat
noiser ids / weights and the workers' commitment rows in pinned host memory.  Reference: the per-worker
commitments and noise a verifier receives (DistSys/main.go:1513-1589, krum.go:227-365).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ..native import hip
from ..utils import streams as S


def _check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"HIP launch of {what} failed (code {err})")


def limits() -> tuple[int, int, int]:
    """(local peer slots, noiser entries per rank, read-back workers) the kernels' argument blocks hold."""
    out = (ctypes.c_int * 3)()
    hip().bsc_vg_limits(out)
    return out[0], out[1], out[2]


class VerifyGather:
    HOST_DEPTH = 4   # the commitment read-back is read lazily (deferred signing: the next round's VRF wait)

    def __init__(self, comm, maxlocal: int, pw: int, nn: int, chunk: int, npairs: int, num_nodes: int, dev):
        self.comm, self.maxlocal, self.pw, self.nn, self.chunk, self.npairs = comm, maxlocal, pw, nn, chunk, npairs
        world = comm.world
        self.gram_bytes = chunk * 256 * 8
        self.commit_off = self.gram_bytes
        self.nz_off = self.commit_off + maxlocal * pw * 4
        self.sc_off = self.nz_off + maxlocal * nn * 4
        self.row_bytes = (self.sc_off + maxlocal * nn * 4 + 15) // 16 * 16
        self.recv = [torch.zeros((world, self.row_bytes), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.gram = torch.empty((max(1, npairs), 256), dtype=torch.float64, device=dev)
        self.nz = torch.empty((world * maxlocal, nn), dtype=torch.int32, device=dev)
        self.sc = torch.empty((world * maxlocal, nn), dtype=torch.float32, device=dev)
        self.host = [torch.empty((num_nodes, pw), dtype=torch.int32, pin_memory=True) for _ in range(self.HOST_DEPTH)]
        self._h = 0
        self.native = None   # NativeSecAgg with the round's own collectives (bsc_round_vg_exchange), else torch's

    @staticmethod
    def fits(maxlocal: int, nn: int, num_nodes: int) -> bool:
        slots, nz, workers = limits()
        return maxlocal <= slots and maxlocal * nn <= nz and num_nodes <= workers

    def gram_out(self, it: int) -> torch.Tensor:
        """This rank's [chunk, 256] Gram slot of iteration it's row (the split Gram kernel writes here)."""
        row = self.recv[it % 2][self.comm.rank]
        return row[: self.gram_bytes].view(torch.float64).view(self.chunk, 256)

    def exchange(self, it: int, commits: torch.Tensor, src_row: list, nz_np: np.ndarray, sc_np: np.ndarray,
                 worker_rows: list):
        """Pack this rank's row, all_gather in place, unpack.  commits int32 [rows, pw] (device) with src_row[j]
        its row of local slot j (-1: none); nz_np / sc_np [maxlocal, nn]; worker_rows: the flat rows of the
        round's workers in plan order.  Returns (gram [npairs, 256], nz, sc [world maxlocal, nn], host commitment
        rows [len(worker_rows), pw] (pinned), event after the read-back)."""
        buf = self.recv[it % 2]
        row = buf[self.comm.rank]
        ml, nn = self.maxlocal, self.nn
        assert commits.dtype == torch.int32 and commits.is_contiguous() and commits.shape[1] == self.pw
        # src_row / worker_rows: int32 numpy arrays (passed by address) or lists
        sr_a = np.ascontiguousarray(src_row, np.int32)
        wr_a = np.ascontiguousarray(worker_rows if len(worker_rows) else [0], np.int32)
        assert sr_a.size == ml
        sr, wr = sr_a.ctypes.data, wr_a.ctypes.data
        nz_c = np.ascontiguousarray(nz_np, np.int32).reshape(-1)
        sc_c = np.ascontiguousarray(sc_np, np.float32).reshape(-1)
        assert nz_c.size == ml * nn and sc_c.size == ml * nn
        host = self.host[self._h]
        self._h = (self._h + 1) % self.HOST_DEPTH
        nw = len(worker_rows)
        na = self.native
        if na is not None:
            # pack, the all_gather in place and unpack in ONE native call (the round's own communicator)
            _check(hip().bsc_round_vg_exchange(na.ctx, it, self.commit_off, self.nz_off, self.sc_off, commits.data_ptr(),
                                               ml, self.pw, sr, nz_c.ctypes.data, sc_c.ctypes.data, ml * nn, self.chunk,
                                               self.npairs, nn, wr, nw, self.gram.data_ptr(), self.nz.data_ptr(),
                                               self.sc.data_ptr(), host.data_ptr(), S.raw()), "round_vg_exchange")
            return self.gram[: self.npairs], self.nz, self.sc, host[:nw], S.record()
        _check(hip().bsc_vg_pack(row.data_ptr(), self.commit_off, self.nz_off, self.sc_off, commits.data_ptr(), ml,
                                 self.pw, sr, nz_c.ctypes.data, sc_c.ctypes.data, ml * nn, S.raw()), "vg_pack")
        self.comm.all_gather_into(buf, row)
        _check(hip().bsc_vg_unpack(buf.data_ptr(), self.row_bytes, self.chunk, self.npairs, self.commit_off,
                                   self.nz_off, self.sc_off, ml, self.pw, nn, self.comm.world, wr, nw,
                                   self.gram.data_ptr(), self.nz.data_ptr(), self.sc.data_ptr(), host.data_ptr(),
                                   S.raw()), "vg_unpack")
        return self.gram[: self.npairs], self.nz, self.sc, host[:nw], S.record()
