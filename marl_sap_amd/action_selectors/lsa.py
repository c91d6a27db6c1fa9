"""Batched scipy-exact linear_sum_assignment on the GPU (asg_lsa_batched, include/asg.h).

Replaces the per-env `scipy.optimize.linear_sum_assignment` loops of the reference
selectors (sap_selectors.py:28-33, :76-91) and env (mock_constellation_env.py:122):
same algorithm, same tie rule, same float64 arithmetic, one wave64 per matrix.
"""
import ctypes

import torch

from .. import _lib


def linear_sum_assignment_batched(C, maximize=False, return_status=False):
    """C: [B, nr, nc] float32/float64 CUDA tensor (any strides).  Returns
    (row_ind, col_ind) int64 [B, min(nr, nc)].  Raises ValueError with scipy's messages
    for invalid/infeasible matrices unless return_status=True (then -1 rows plus a
    status tensor: 0 ok, -4 invalid entries, -5 infeasible)."""
    if not C.is_cuda:
        raise ValueError("linear_sum_assignment_batched needs a CUDA (ROCm) tensor")
    if C.dim() == 2:
        C = C.unsqueeze(0)
    if C.dtype not in (torch.float32, torch.float64):
        C = C.to(torch.float64)
    B, nr, nc = C.shape
    k = min(nr, nc)
    row = torch.empty((B, k), dtype=torch.int64, device=C.device)
    col = torch.empty((B, k), dtype=torch.int64, device=C.device)
    status = torch.empty((B,), dtype=torch.int32, device=C.device)
    with torch.cuda.device(C.device):
        _lib.check(_lib.lib().asg_lsa_batched(
            ctypes.c_void_p(C.data_ptr()), _lib.dtype_code(C.dtype), _lib.i64arr(C.stride()), B, nr, nc,
            int(bool(maximize)), ctypes.c_void_p(row.data_ptr()), ctypes.c_void_p(col.data_ptr()),
            ctypes.c_void_p(status.data_ptr()), _lib.stream_ptr(C.device)))
    if return_status:
        return row, col, status
    raise_on_status(status)
    return row, col


def raise_on_status(status):
    """Raise the reference's scipy error for the first failed matrix (syncs)."""
    if status.numel() == 0:
        return
    code = int(status.min().item())  # error codes are negative
    if code == 0:
        return
    if code == _lib.ASG_E_LSA_INVALID:
        raise ValueError("matrix contains invalid numeric entries")
    if code == _lib.ASG_E_LSA_INFEASIBLE:
        raise ValueError("cost matrix is infeasible")
    raise RuntimeError(f"LSA failed (status {code})")


class DeferredStatus:
    """Accumulates LSA status on the device so the rollout loop never syncs per step;
    `flush()` (called by the runner once per episode) raises the minimum status seen (error
    codes are negative: the most negative, not necessarily the first).  `sticky(B)`: a zeroed
    per-env int32 word that kernels min-accumulate into themselves
    (asg_sap_select_into) -- no reduction launches per call."""

    def __init__(self):
        self._acc = None
        self._sticky = None

    def add(self, status):
        m = status.min() if status.numel() else None
        if m is None:
            return
        self._acc = m if self._acc is None else torch.minimum(self._acc, m)

    def sticky(self, B, device):
        st = self._sticky
        if st is None or st.numel() != B or st.device != device:
            if st is not None:
                self.add(st)  # keep what the old buffer holds
            st = self._sticky = torch.zeros(B, dtype=torch.int32, device=device)
        return st

    def flush(self):
        if self._sticky is not None:
            self.add(self._sticky)
            self._sticky = None
        acc, self._acc = self._acc, None
        if acc is not None:
            raise_on_status(acc.reshape(1))
