"""Batched LSA targets for the SAP Q-learners.

The reference computes the SAP target of every (episode, t) with a serial scipy loop on
the CPU (learners/sap_q_learner.py:86-108; learners/filtered_sap_q_learner.py:115-133):

    target_mac_out[avail_actions[:, 1:] == 0] = -9999
    for bn, t:  row, col = linear_sum_assignment(C[bn, t], maximize=True)
                target_max_qvals[bn, t, :] = target_mac_out[bn, t, row, col]

with C = target_mac_out (or, with double_q, the live mac_out masked the same way at
t + 1).  Here the B x (T-1) problems are one `asg_lsa_batched` launch (same algorithm,
same tie rule, f32 costs widened exactly as scipy's float64 conversion does) and the
gather stays on the device: no host copies, no Python loop.
"""
import torch

from ..action_selectors.lsa import linear_sum_assignment_batched


def sap_target_max_qvals(target_mac_out, avail_actions, mac_out=None, double_q=False, mask_value=-9999.0):
    """target_mac_out: [B, T-1, n, m] target-network Q-values for t = 1 .. T-1;
    avail_actions: [B, T, n, m]; mac_out: [B, T, n, m] live Q-values (double_q only).
    Returns target_max_qvals [B, T-1, n] (float32, on the device).  mask_value: -9999 as
    sap_q_learner.py:89, -9999999 as filtered_sap_q_learner.py:115."""
    B, T1, n, m = target_mac_out.shape
    if n > m:
        # the reference assigns min(n, m) values into n slots (a broadcast error there)
        raise ValueError("SAP targets need n <= m (one task per agent)")
    unavailable = avail_actions[:, 1:] == 0
    tgt = target_mac_out.detach().masked_fill(unavailable, mask_value)
    if double_q:
        if mac_out is None:
            raise ValueError("double_q needs the live mac_out")
        cost = mac_out.detach()[:, 1:].masked_fill(unavailable, mask_value)
    else:
        cost = tgt
    flat = tgt.reshape(B * T1, n, m)
    row, col = linear_sum_assignment_batched(cost.reshape(B * T1, n, m), maximize=True)
    vals = flat[torch.arange(B * T1, device=flat.device).unsqueeze(1), row, col]
    out = torch.zeros((B, T1, n), dtype=torch.float32, device=flat.device)
    out.view(B * T1, n)[:, : row.shape[1]] = vals.to(torch.float32)
    return out
