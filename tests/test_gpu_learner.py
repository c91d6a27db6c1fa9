"""batched LSA targets for the SAP Q-learners against the reference's
own serial scipy loop (learners/sap_q_learner.py:86-108), restated here on CPU copies of
the same tensors.  Values are gathered, not computed, so agreement is bit-exact."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
scipy_opt = pytest.importorskip("scipy.optimize")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.learners import sap_target_max_qvals  # noqa: E402

DEV = torch.device("cuda", 0)


def reference_targets(target_mac_out, avail_actions, mac_out, double_q, mask_value):
    """sap_q_learner.py:86-108 (scipy loop on the CPU)."""
    target_mac_out = target_mac_out.clone().cpu()
    avail_actions = avail_actions.cpu()
    target_mac_out[avail_actions[:, 1:] == 0] = mask_value
    B, T1, n, m = target_mac_out.shape
    out = torch.zeros((B, T1, n))
    if double_q:
        live = mac_out.clone().detach().cpu()
        live[avail_actions == 0] = mask_value
        for bn in range(B):
            for t in range(1, T1 + 1):
                r, c = scipy_opt.linear_sum_assignment(live[bn, t].numpy(), maximize=True)
                out[bn, t - 1, :] = target_mac_out[bn, t - 1, r, c]
    else:
        for bn in range(B):
            for t in range(T1):
                r, c = scipy_opt.linear_sum_assignment(target_mac_out[bn, t].numpy(), maximize=True)
                out[bn, t, :] = target_mac_out[bn, t, r, c]
    return out


@pytest.mark.parametrize("B,T,n,m,double_q,ties,mask_value", [
    (4, 7, 5, 9, False, False, -9999.0), (4, 7, 5, 9, True, False, -9999.0),
    (3, 6, 8, 8, False, True, -9999.0), (3, 6, 8, 8, True, True, -9999999.0),
    (8, 21, 64, 64, False, False, -9999.0), (2, 5, 1, 3, True, True, -9999.0)])
def test_sap_targets_match_scipy_loop(B, T, n, m, double_q, ties, mask_value):
    g = torch.Generator().manual_seed(B * 1000 + T * 10 + n)
    q_t = torch.randn((B, T - 1, n, m), generator=g)
    q_live = torch.randn((B, T, n, m), generator=g)
    if ties:  # coarse values: many equal costs, exercising scipy's tie rule
        q_t, q_live = (q_t * 2).round() / 2, (q_live * 2).round() / 2
    avail = torch.rand((B, T, n, m), generator=g) > 0.3
    avail |= torch.eye(n, m, dtype=torch.bool)  # keep every row feasible
    ref = reference_targets(q_t, avail, q_live, double_q, mask_value)
    got = sap_target_max_qvals(q_t.to(DEV), avail.to(DEV), q_live.to(DEV), double_q=double_q,
                               mask_value=mask_value)
    assert got.dtype == torch.float32 and got.shape == (B, T - 1, n)
    assert torch.equal(got.cpu(), ref)


def test_sap_targets_reject_more_agents_than_tasks():
    with pytest.raises(ValueError):
        sap_target_max_qvals(torch.zeros((1, 2, 5, 3), device=DEV), torch.ones((1, 3, 5, 3), device=DEV))
