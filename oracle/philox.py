"""numpy restatement of the product's counter-based draws (TEST INFRASTRUCTURE ONLY).

Philox4x32-10 (Salmon et al., SC'11) exactly as marl_sap_amd/csrc/asg_device.h
`philox4x32_10` computes it, and the epsilon-greedy selection draw built on it
(asg_agent.hip `select_finish`, asg_select.hip): the row's counter is
(global row lo, global row hi, kCtrSelect, call counter) under the selector key
(k0, k1) = (seed lo, seed hi ^ 0x5bd1e995); the row explores when
(x >> 8) * 2^-24 < epsilon and then takes the target-th available task,
target = (y * count) >> 32.  The reference draws these from torch's CPU generator
(classic_selectors.py:45-52), which no GPU kernel can reproduce; this restatement lets
a test predict every exploring row of a GPU rollout and check the rest against a
greedy argmax of the PyTorch RNNAgent.
"""
import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)
K_CTR_SELECT = 6


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays (broadcast); returns (x, y, z, w)."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint64) & _MASK for v in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + _W0) & 0xFFFFFFFF
        k1 = (k1 + _W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def select_keys(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, ((seed >> 32) ^ 0x5BD1E995) & 0xFFFFFFFF


def eps_greedy_draws(seed, global_rows, counter, epsilon, n_avail):
    """(explore mask, target index among the available tasks) of the fused / standalone
    epsilon-greedy selection for the given global (env, agent) rows at one call counter."""
    rows = np.asarray(global_rows, dtype=np.uint64)
    k0, k1 = select_keys(seed)
    x, y, _, _ = philox4x32_10(rows & _MASK, rows >> np.uint64(32), K_CTR_SELECT, counter, k0, k1)
    u = (x >> np.uint64(8)).astype(np.float32) * np.float32(5.9604644775390625e-08)
    explore = u < np.float32(epsilon) if epsilon > 0 else np.zeros(rows.shape, bool)
    target = ((y * np.asarray(n_avail, dtype=np.uint64)) >> np.uint64(32)).astype(np.int64)
    return explore, target
