"""Host model of the SAP selector's two LSA solvers (CPU, numpy; no GPU):

    python tools/lsa_fastpath_sim.py [--problems 4] [--seed 3]

For SAP-selector matrices (Q of a random-init RNNAgent on the mock env's observations from
the C oracle env, plus the selector's Gaussian noise of std 2 eps mean|Q|) and for uniform
matrices, it counts the augmenting-path steps of
  * scipy's algorithm (every row's Dijkstra from u = v = 0; csrc/lsa_wave.h lsa_solve_reg64),
  * the certified fast path (csrc/lsa_wave.h lsa_fast_reg64): row + column reduction, then the
    same shortest-augmenting-path step for the rows it leaves free only,
checks both assignments against scipy, and evaluates the fast path's uniqueness certificate
(dual feasibility within S 2^-40, acyclic near-tight graph at S 2^-30).  --q-seq: the warm start
(asg_sap_select_warm) against the cold one on captured consecutive Q (tools/sap_reda_probe.py).  The kernel's steps
and certificate are this model's; the GPU figures are bench.py's roofline_lsa.
"""
import argparse
import os
import sys
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

INF = float("inf")


def scipy_steps(C):
    """scipy 1.15.3's shortest augmenting path (rectangular_lsap.cpp), counting steps."""
    n, m = C.shape
    u, v = np.zeros(n), np.zeros(m)
    r4c, c4r, path = -np.ones(m, int), -np.ones(n, int), -np.ones(m, int)
    steps = 0
    for cur in range(n):
        spc = np.full(m, INF)
        rem = list(range(m - 1, -1, -1))
        SR, SC = np.zeros(n, bool), np.zeros(m, bool)
        i, minv, sink = cur, 0.0, -1
        while sink == -1:
            steps += 1
            SR[i] = True
            idx, lowest = -1, INF
            for it, j in enumerate(rem):
                r = minv + C[i, j] - u[i] - v[j]
                if r < spc[j]:
                    path[j], spc[j] = i, r
                if spc[j] < lowest or (spc[j] == lowest and r4c[j] == -1):
                    lowest, idx = spc[j], it
            minv = lowest
            j = rem[idx]
            if r4c[j] == -1:
                sink = j
            else:
                i = r4c[j]
            SC[j] = True
            rem[idx] = rem[-1]
            rem.pop()
        u[cur] += minv
        for i2 in range(n):
            if SR[i2] and i2 != cur:
                u[i2] += minv - spc[c4r[i2]]
        v[SC] -= minv - spc[SC]
        j = sink
        while True:
            i2 = path[j]
            r4c[j] = i2
            c4r[i2], j = j, c4r[i2]
            if i2 == cur:
                break
    return c4r, steps


def fast_path(C, vwarm=None, return_v=False):
    """lsa_fast_reg64: (assignment, steps, certified[, final v]).  vwarm: the warm start's
    column duals (u_k = min_j (c_kj - vwarm_j), then the same column reduction and claims)."""
    n = C.shape[0]
    u = C.min(1).copy() if vwarm is None else (C - vwarm[None, :]).min(1)  # row reduction
    R = C - u[:, None]
    v = R.min(0).copy()  # column reduction of the rest
    imin = R.argmin(0)
    x, y = -np.ones(n, int), -np.ones(n, int)
    for i in range(n):  # each row keeps the lowest column whose minimum it holds
        js = np.where(imin == i)[0]
        if len(js):
            x[i], y[js[0]] = js[0], i
    path = -np.ones(n, int)
    steps = 0
    for cur in [i for i in range(n) if x[i] < 0]:
        spc = np.full(n, INF)
        rem = np.ones(n, bool)
        i, minv, sink = cur, 0.0, -1
        while sink == -1:
            steps += 1
            r = ((minv + C[i]) - u[i]) - v
            upd = rem & (r < spc)
            spc[upd], path[upd] = r[upd], i
            tie = np.where(rem & (spc == minv))[0]  # still at the current distance: no reduction
            if len(tie):
                cand, lowest = tie, minv
            else:
                key = np.where(rem, spc, INF)
                lowest = key.min()
                cand = np.where(key == lowest)[0]
            j = int(cand[0])
            minv = lowest
            rem[j] = False
            if y[j] == -1:
                sink = j
            else:
                i = y[j]
        sc = ~rem
        for r2 in range(n):
            if r2 == cur:
                u[r2] += minv
            elif x[r2] >= 0 and sc[x[r2]]:
                u[r2] += minv - spc[x[r2]]
        v[sc] -= minv - spc[sc]
        j = sink
        while True:
            pi = path[j]
            y[j] = pi
            x[pi], j = j, x[pi]
            if pi == cur:
                break
    rc = (C - u[:, None]) - v[None, :]
    S = np.abs(C).max() + np.abs(u).max() + np.abs(v).max()
    tight, slack = S * 2.0 ** -30, S * 2.0 ** -40
    ok = rc.min() >= -slack and np.abs(rc[np.arange(n), x]).max() <= slack
    adj = np.zeros((n, n), bool)  # column x_i -> column j over near-tight edges
    for i in range(n):
        for j in np.where(rc[i] <= tight)[0]:
            if j != x[i]:
                adj[x[i], j] = True
    A = np.ones(n, bool)
    while A.any():
        nA = A & (adj & A[None, :]).any(1)
        if (nA == A).all():
            break
        A = nA
    if return_v:
        return x, steps, bool(ok and not A.any()), v
    return x, steps, bool(ok and not A.any())


def sap_matrices(n, m, count, use_rnn, eps, seed):
    import torch
    from oracle import oracle as ora
    from marl_sap_amd.modules.agents.rnn_agent import RNNAgent
    from scipy.optimize import linear_sum_assignment
    torch.manual_seed(seed)
    agent = RNNAgent(m * 4, SimpleNamespace(m=m, hidden_dim=64, use_rnn=use_rnn))
    out = []
    for e in range(count):
        env = ora.OracleMockEnv(n, m, 20, 3, 0.5, seed=seed * 1000 + e)
        obs = env.reset()
        h = torch.zeros(n, 64)
        rng = np.random.RandomState(e)
        for _ in range(3):
            with torch.no_grad():
                q, h = agent(torch.tensor(obs, dtype=torch.float32), h)
            q = q.numpy().astype(np.float32)
            out.append((q + rng.randn(n, m).astype(np.float32) * np.float32(2 * eps * np.abs(q).mean()))
                       .astype(np.float32))
            env.step(linear_sum_assignment(out[-1], maximize=True)[1])
            obs = env._obs
    return out


def warm_sequence(path, eps, seed=0, envs=16):
    """Cold vs warm-started fast path on consecutive selections of captured Q sequences
    ([steps, envs, n, n] float32, tools/sap_reda_probe.py --save): each warm call starts from the
    previous step's final column duals (shifted to a zero minimum, as the kernel keeps them)."""
    from scipy.optimize import linear_sum_assignment
    Q = np.load(path)
    rng = np.random.RandomState(seed)
    tc = tw = cc = cw = 0
    for e in range(min(envs, Q.shape[1])):
        vprev = None
        for t in range(Q.shape[0]):
            q = Q[t, e].astype(np.float32)
            q = (q + rng.randn(*q.shape).astype(np.float32) * np.float32(2 * eps * np.abs(q).mean())).astype(np.float32)
            C = -q.astype(np.float64)
            ref = linear_sum_assignment(q, maximize=True)[1]
            xc, sc, okc, vc = fast_path(C, return_v=True)
            xw, sw, okw, vw = fast_path(C, vwarm=vprev, return_v=True)
            assert (xc == ref).all() and (xw == ref).all()
            if vprev is not None:
                tc, tw, cc, cw = tc + sc, tw + sw, cc + okc, cw + okw
            vprev = vw - vw.min()
    print(f"{os.path.basename(path)} eps={eps}: cold {tc} steps, warm {tw} ({tw / max(tc, 1):.2f}x); certified "
          f"cold {cc}, warm {cw}")


def main():
    from scipy.optimize import linear_sum_assignment
    p = argparse.ArgumentParser()
    p.add_argument("--problems", type=int, default=4)
    p.add_argument("--seed", type=int, default=3)
    p.add_argument("--q-seq", nargs="*", default=[], help="captured Q sequences (.npy) for the warm-start model")
    p.add_argument("--eps", type=float, default=0.0)
    a = p.parse_args()
    if a.q_seq:
        for path in a.q_seq:
            warm_sequence(path, a.eps)
        return
    for eps in (0.0, 0.05, 0.3, 1.0):
        for rnn in (False, True):
            mats = sap_matrices(64, 64, a.problems, rnn, eps, a.seed)
            ts = tf = cert = 0
            for Q in mats:
                C = -Q.astype(np.float64)
                ref = linear_sum_assignment(Q, maximize=True)[1]
                xa, sa = scipy_steps(C)
                xb, sb, ok = fast_path(C)
                assert (xa == ref).all() and (xb == ref).all()
                ts, tf, cert = ts + sa, tf + sb, cert + ok
            k = len(mats)
            print(f"SAP Q eps={eps:<4} {'GRU   ' if rnn else 'Linear'}: scipy {ts / k:6.0f} steps, fast path "
                  f"{tf / k:6.0f} ({tf / ts:.2f}x), certified {cert}/{k}")
    rng = np.random.RandomState(a.seed)
    mats = [rng.rand(64, 64) for _ in range(8)]
    ts = sum(scipy_steps(-Q)[1] for Q in mats)
    tf = sum(fast_path(-Q)[1] for Q in mats)
    print(f"uniform 64x64: scipy {ts / 8:.0f} steps, fast path {tf / 8:.0f} ({tf / ts:.2f}x)")


if __name__ == "__main__":
    main()
