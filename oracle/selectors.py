"""CPU ORACLE for the filtered selectors and HAALSelector (test infrastructure only:
imported by tests/ alone; the product never imports oracle/).

Plain numpy restatements with the scipy-exact LSA of asg_oracle.c (oracle.lsa), pinned
by tests/test_oracle_golden.py against tests/golden/filtered_selectors.npz and
tests/golden/haal.npz (generated from the reference by tests/golden/make_golden.py).
The random draws of the reference (torch.rand_like tie noise, torch.normal exploration
noise) are inputs here, so a restatement fed the reference's recorded draws must
reproduce its actions exactly.
"""
import numpy as np

from . import oracle as ora


def total_beta_f16(beta):
    """beta.sum(-1) of a float16 tensor as torch computes it: float32 accumulation left
    to right, rounded to float16 (filtered_sap_selectors.py:24, filtered_classic_selectors.py:21)."""
    b = np.asarray(beta)
    if b.dtype != np.float16:
        return b.sum(-1)
    acc = np.zeros(b.shape[:-1], dtype=np.float32)
    for l in range(b.shape[-1]):
        acc = acc + b[..., l].astype(np.float32)
    return acc.astype(np.float16)


def top_m(beta, M):
    """th.topk(total_beta, k=M).indices with ties to the lower index (torch leaves the tie
    order unspecified; the reference fixtures are tie-free at the top-M boundary)."""
    tot = total_beta_f16(beta).astype(np.float64)
    return np.argsort(-tot, axis=-1, kind="stable")[..., :M]


def benefit_matrix(q, beta, M, tie_noise):
    """The filtered selectors' [B, n, m] matrix (filtered_sap_selectors.py:37-55): the
    baseline Q (column M) plus float32(u * 1e-8), then the top-M Q-values scattered onto
    each agent's top-M tasks."""
    q = np.asarray(q, dtype=np.float32)
    B, n, _ = q.shape
    m = beta.shape[2]
    base = np.broadcast_to(q[:, :, M:M + 1], (B, n, m)).astype(np.float32)
    mat = base + np.asarray(tie_noise, dtype=np.float32) * np.float32(1e-8)
    top = top_m(beta, M)
    bi, ii = np.indices(top.shape[:2])
    mat[bi[..., None], ii[..., None], top] = q[:, :, :M]
    return mat


def filtered_sap(q, beta, M, tie_noise, gauss_noise=None):
    """FilteredSAPActionSelector / the test-mode FilteredEpsGrSAPTestActionSelector
    (filtered_sap_selectors.py:35-62, :100-115): LSA(maximize) per env of the matrix plus
    the (given) Gaussian noise; float32 task ids."""
    mat = benefit_matrix(q, beta, M, tie_noise)
    if gauss_noise is not None:
        mat = mat + np.asarray(gauss_noise, dtype=np.float32)
    out = np.zeros(mat.shape[:2], dtype=np.float32)
    for b in range(mat.shape[0]):
        out[b] = ora.lsa(mat[b].astype(np.float64), maximize=True)[1]
    return out


def filtered_greedy(q, beta, M, tie_noise):
    """The epsilon = 0 action of FilteredEpsilonGreedyActionSelector /
    FilteredEpsGrSAPTestActionSelector (train): first maximal index of each matrix row
    (torch.max order, no availability mask -- filtered_classic_selectors.py:57-61)."""
    mat = benefit_matrix(q, beta, M, tie_noise)
    return np.argmax(mat, axis=-1).astype(np.int64)


# ---------------------------------------------------------------------------------------
# HAALSelector (non_rl_selectors.py:54-118) on RealConstellationEnv with constant benefits
# ---------------------------------------------------------------------------------------
def time_interval_sequences(L):
    """build_time_interval_sequences(generate_all_time_intervals(L), L) (utils/methods.py:
    309-349): every composition of [0, L) into consecutive intervals, depth first with the
    shorter first interval first."""
    out = []

    def rec(seq, last):
        if last == L - 1:
            out.append(tuple(seq))
            return
        for j in range(last + 1, L):
            rec(seq + [(last + 1, j)], j)

    rec([], -1)
    return out


def real_beta(table, prios, k, L, T):
    """RealConstellationEnv.beta at step k (real_constellation_env.py:127, :167-170):
    table[:, :, k:k+L] * prios, zero past T."""
    n, m, _ = table.shape
    cur = np.zeros((n, m, L))
    eff = max(0, min(L, T - k))
    cur[:, :, :eff] = table[:, :, k:k + eff]
    return cur * np.asarray(prios)[None, :, None]


def real_beta_hat(beta, prev, lam, T_trans):
    """RealConstellationEnv.beta_hat (:282-327) for one state: penalty on the l = 0 slice."""
    n, m, _ = beta.shape
    pam = np.zeros((n, m))
    pam[np.arange(n), prev] = 1
    pen = (pam @ T_trans) * (beta.sum(-1) > 1e-12)
    bh = beta.copy()
    bh[:, :, 0] = bh[:, :, 0] - lam * pen
    return bh


def real_rewards(beta, prev, a, lam, T_trans):
    """RealConstellationEnv.step rewards (:145-160)."""
    n, m, _ = beta.shape
    cnt = np.zeros(m)
    for i in range(n):
        cnt[a[i]] += 1
    bh = real_beta_hat(beta, prev, lam, T_trans)
    r = []
    for i in range(n):
        v = bh[i, a[i], 0]
        r.append(v / cnt[a[i]] if v > 0 else v)
    return r


def haal(table, prios, T_trans, lam, k, prev, L, T):
    """HAALSelector for one env at step k with previous assignments `prev`: returns
    (action, values per time-interval sequence).  Each sequence forks the env, and per
    interval takes LSA(maximize) of beta_hat summed over L and steps it interval-length
    times; the action is the first interval's assignment of the best sequence (strict >,
    first wins)."""
    eff = min(L, T - k)
    seqs = time_interval_sequences(eff)
    best, best_a, vals = -np.inf, None, []
    for tis in seqs:
        kk, pv, tot, first = k, np.asarray(prev), 0, None
        for ti in tis:
            beta = real_beta(table, prios, kk, L, T)
            bh = real_beta_hat(beta, pv, lam, T_trans)
            a = ora.lsa(bh.sum(axis=-1), maximize=True)[1]
            if first is None:
                first = a
            for _ in range(ti[1] - ti[0] + 1):
                beta = real_beta(table, prios, kk, L, T)
                tot += sum(real_rewards(beta, pv, a, lam, T_trans))
                kk, pv = kk + 1, a
        vals.append(tot)
        if tot > best:
            best, best_a = tot, first
    return best_a, np.array(vals)


def variant_beta_hat(kind, beta, prev, lam, T_trans, power):
    """RealPowerConstellationEnv.beta_hat (real_power_constellation_env.py:310-352) /
    InterferenceConstellationEnv.beta_hat (interference_constellation_env.py:355-406, its penalty
    mask is 1 - I whatever T_trans) for one state: the plain beta_hat, rows of satellites below
    1e-12 power zeroed."""
    n, m, _ = beta.shape
    tt = np.ones((m, m)) - np.eye(m) if kind == "interference" else T_trans
    bh = real_beta_hat(beta, prev, lam, tt)
    dead = np.asarray(power) < 1e-12
    bh[dead] = 0.0
    return bh


def variant_rewards(kind, beta, prev, a, lam, T_trans, power, bands=None, nbr=None):
    """One step's rewards: RealPowerConstellationEnv.step (:145-165) or
    InterferenceConstellationEnv.interference_reward_function (:309-353)."""
    n, m, _ = beta.shape
    power = np.asarray(power)
    if kind == "power":
        cnt = np.zeros(m)
        for i in range(n):
            cnt[a[i]] += 1
        bh = variant_beta_hat(kind, beta, prev, lam, T_trans, power)
        r = []
        for i in range(n):
            if power[i] > 0:
                v = bh[i, a[i], 0]
                r.append(v / cnt[a[i]] if v > 0 else v)
            else:
                r.append(0)
        return r
    app = np.where(power <= 0, 0, 1) * np.where(beta[:, :, 0][np.arange(n), a] < 1e-12, 0, 1)
    cnt = np.zeros(m)
    for i in range(n):
        if app[i] == 1:
            cnt[a[i]] += 1
    r = []
    for i in range(n):
        same = [j for j in range(n) if bands[j] == bands[i]]
        conflicts = np.sum(nbr[a[i], a[same]] * app[same]) - 1
        v = beta[i, a[i], 0] * 0.5 ** conflicts
        if cnt[a[i]] > 0:
            v /= cnt[a[i]]
        if app[i] and prev[i] != a[i]:
            v -= lam
        r.append(v)
    return r


def power_update(beta, a, power):
    """The power drain / recharge of one step (real_power_constellation_env.py:170-178)."""
    p = np.array(power, dtype=np.float64)
    for i in range(len(p)):
        if p[i] > 0:
            if beta[i, a[i], 0] > 1e-12:
                p[i] -= 0.2
            else:
                p[i] = min(p[i] + 0.1, 1)
    return p


def haal_variant(kind, table, prios, T_trans, lam, k, prev, power, L, T, bands=None, nbr=None):
    """HAALSelector (non_rl_selectors.py:54-118) over a power / interference env at step k with
    previous assignments `prev` and power states `power`: each sequence forks the env (power
    included), per interval LSA(maximize) of beta_hat (power-zeroed) summed over L, stepped
    interval-length times with the variant's rewards and power updates.  Returns (action,
    values per sequence)."""
    eff = min(L, T - k)
    seqs = time_interval_sequences(eff)
    best, best_a, vals = -np.inf, None, []
    for tis in seqs:
        kk, pv, pw, tot, first = k, np.asarray(prev), np.array(power, dtype=np.float64), 0, None
        for ti in tis:
            beta = real_beta(table, prios, kk, L, T)
            bh = variant_beta_hat(kind, beta, pv, lam, T_trans, pw)
            a = ora.lsa(bh.sum(axis=-1), maximize=True)[1]
            if first is None:
                first = a
            for _ in range(ti[1] - ti[0] + 1):
                beta = real_beta(table, prios, kk, L, T)
                tot += sum(variant_rewards(kind, beta, pv, a, lam, T_trans, pw, bands, nbr))
                pw = power_update(beta, a, pw)
                kk, pv = kk + 1, a
        vals.append(tot)
        if tot > best:
            best, best_a = tot, first
    return best_a, np.array(vals)
