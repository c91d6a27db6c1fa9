"""Pins the CPU oracle (oracle/) against the golden vectors captured from the reference
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest


def test_mt19937_words(golden, oracle):
    g = golden("mt19937_words")
    for s, words in zip(g["seeds"], g["words"]):
        mt = oracle.MT(int(s))
        np.testing.assert_array_equal(mt.next32(len(words)), words)


def test_mt19937_derived(golden, oracle):
    g = golden("mt19937_words")
    mt = oracle.MT(3)
    np.testing.assert_array_equal(np.array([mt.rand() for _ in range(50)]), g["rand_seed3"])
    mt = oracle.MT(3)
    np.testing.assert_array_equal(np.array([mt.uniform(0, 20) for _ in range(25)]),
                                  g["uniform0_20_seed3"])
    for m, perm in zip(g["perm_sizes"], g["perms"]):
        np.testing.assert_array_equal(oracle.MT(int(m)).permutation(int(m)), perm[:m])


def _table_close(a, b):
    """Benefit tables are the same float64 expression of the same MT19937 draws; the
    only inexact op is exp.  numpy's AVX-512 float64 exp is not correctly rounded (its
    error grows with |argument|: up to ~1e-13 relative for arguments near -150), while
    the oracle uses libm's, so float64 values agree to rtol 1e-12; the zero pattern and
    the float32 values the EpisodeBatch stores are identical."""
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=0)
    np.testing.assert_array_equal(a == 0, b == 0)
    np.testing.assert_array_equal(a.astype(np.float32), b.astype(np.float32))


def test_mock_construct_reset(golden, oracle):
    g = golden("mock_reset")
    for c in range(int(g["n_cases"])):
        n, m, T, L, s = [int(x) for x in g[f"c{c}_shape"]]
        mt = oracle.MT(s)
        env = oracle.OracleMockEnv(n, m, T, L, 0.5, mt=mt)
        _table_close(env.sat_prox_mat, g[f"c{c}_init_table"])
        env.reset()
        _table_close(env.sat_prox_mat, g[f"c{c}_table"])
        np.testing.assert_array_equal(env.prev_assigns, g[f"c{c}_prev_assigns"])
        _table_close(env._obs, g[f"c{c}_obs"])
        _table_close(env.beta, g[f"c{c}_beta"])
        key, pos = mt.state()
        assert pos == int(g[f"c{c}_mt_pos_after"])
        np.testing.assert_array_equal(key, g[f"c{c}_mt_key_after"])


def test_mock_steps(golden, oracle):
    g = golden("mock_step")
    for c in range(int(g["n_cases"])):
        n, m, T, L = [int(x) for x in g[f"c{c}_spec"]]
        lam = float(g[f"c{c}_lambda"])
        kind = str(g[f"c{c}_kind"])
        bids = kind.startswith("bids")
        mt = oracle.MT(100 + c)
        if kind != "dense":  # the fixture drew its table from the global stream first
            tab = oracle.generate(mt, n, m, T, 3.0, 6.0)
            keep = np.ones_like(tab, dtype=bool)
            keep[0, 0], keep[0, 1], keep[1, 1] = False, False, False
            np.testing.assert_allclose(tab[keep], g[f"c{c}_table"][keep], rtol=1e-12, atol=0)
        env = oracle.OracleMockEnv(n, m, T, L, lam, bids_as_actions=bids,
                                   sat_prox_mat=g[f"c{c}_table"], mt=mt)
        env.reset()
        np.testing.assert_array_equal(env.prev_assigns, g[f"c{c}_prev0"])
        np.testing.assert_array_equal(env._obs, g[f"c{c}_obs0"])
        for t in range(T):
            r, d, info = env.step(g[f"c{c}_actions"][t])
            np.testing.assert_array_equal(np.array(r), g[f"c{c}_rewards"][t], err_msg=f"{c},{t}")
            np.testing.assert_array_equal(env._obs, g[f"c{c}_obs"][t])
            np.testing.assert_array_equal(env.beta, g[f"c{c}_beta"][t])
            np.testing.assert_array_equal(env.prev_assigns, g[f"c{c}_prev"][t])
            assert d == bool(g[f"c{c}_done"][t])


def test_beta_hat(golden, oracle):
    g = golden("mock_step")
    out = oracle.beta_hat(g["bh_beta"], g["bh_prev"], float(g["bh_lambda"]), g["bh_T_trans"])
    np.testing.assert_array_equal(out, g["bh_out"])
    out2 = oracle.beta_hat(g["bh_beta"][0], g["bh_prev"][0], float(g["bh_lambda"]), g["bh_T_trans"])
    np.testing.assert_array_equal(out2, g["bh_out2d"])


def test_lsa(golden, oracle):
    g = golden("lsa")
    for k in range(int(g["n_cases"])):
        r, c = oracle.lsa(g[f"k{k}_C"], bool(g[f"k{k}_max"]))
        np.testing.assert_array_equal(r, g[f"k{k}_row"], err_msg=str(k))
        np.testing.assert_array_equal(c, g[f"k{k}_col"], err_msg=str(k))
    for e in range(int(g["n_err"])):
        msg = str(g[f"e{e}_msg"])
        with pytest.raises(ValueError, match=msg):
            oracle.lsa(g[f"e{e}_C"], bool(g[f"e{e}_max"]))


def test_real_env_oracle_matches_reference_fixture(golden, oracle):
    """RealConstellationEnv restatement (oracle/asg_real_oracle.c) vs the reference's own
    reset/step outputs on tie-free injected tables: float64 bit-exact."""
    d = golden("real_env")
    for c in range(int(d["n_cases"])):
        n, m, T, L, N, M = (int(x) for x in d[f"r{c}_spec"])
        env = oracle.OracleRealEnv(d[f"r{c}_table"], N, M, L, float(d[f"r{c}_lambda"]),
                                   T_trans=d[f"r{c}_T_trans"], task_prios=d[f"r{c}_prios"])
        assert env.obs_size == int(d[f"r{c}_obs_size"])
        obs0 = env.reset()
        np.testing.assert_array_equal(obs0, d[f"r{c}_obs0"])
        np.testing.assert_array_equal(env.beta, d[f"r{c}_beta0"])
        np.testing.assert_array_equal(env.prev_assigns, d[f"r{c}_prev0"])
        for t in range(T):
            r, done, _ = env.step(d[f"r{c}_actions"][t])
            np.testing.assert_array_equal(r, d[f"r{c}_rewards"][t])
            np.testing.assert_array_equal(env.obs, d[f"r{c}_obs"][t])
            np.testing.assert_array_equal(env.beta, d[f"r{c}_beta"][t])
            np.testing.assert_array_equal(env.prev_assigns, d[f"r{c}_prev"][t])
            assert done == bool(d[f"r{c}_done"][t])


def test_real_variant_oracle_matches_reference_fixture(golden, oracle):
    """RealPowerConstellationEnv / InterferenceConstellationEnv restatement vs the
    reference's own outputs (power drain and death, band conflicts, handovers)."""
    d = golden("real_variants")
    for c in range(int(d["n_cases"])):
        n, m, T, L, N, M = (int(x) for x in d[f"v{c}_spec"])
        env = oracle.OracleRealVariantEnv(str(d[f"v{c}_kind"]), d[f"v{c}_table"], N, M, L, float(d[f"v{c}_lambda"]),
                                          d[f"v{c}_prios"], d[f"v{c}_prev0"], bands=d[f"v{c}_bands"],
                                          neighbor_matrix=d[f"v{c}_nbr"])
        assert env.obs_size == int(d[f"v{c}_obs_size"])
        np.testing.assert_array_equal(env.reset(), d[f"v{c}_obs0"])
        np.testing.assert_array_equal(env.beta, d[f"v{c}_beta0"])
        for t in range(T):
            r, done, _ = env.step(d[f"v{c}_actions"][t])
            np.testing.assert_array_equal(r, d[f"v{c}_rewards"][t])
            np.testing.assert_array_equal(env.power_states, d[f"v{c}_power"][t])
            np.testing.assert_array_equal(env.obs, d[f"v{c}_obs"][t])
            np.testing.assert_array_equal(env.beta, d[f"v{c}_beta"][t])
            np.testing.assert_array_equal(env.prev_assigns, d[f"v{c}_prev"][t])
            assert done == bool(d[f"v{c}_done"][t])


# ---- round 2: filtered selectors, HAALSelector (oracle/selectors.py) -------------------
def test_f16_total_beta_matches_torch(golden):
    """The oracle's float16 L-sum is torch's Half sum (float32 accumulation, one rounding)."""
    import torch
    from oracle.selectors import total_beta_f16
    g = golden("filtered_selectors")
    for c in g["cases"]:
        beta = g[f"{c}__beta"]
        np.testing.assert_array_equal(total_beta_f16(beta), torch.from_numpy(beta).sum(-1).numpy())


def test_filtered_selectors_oracle(golden, oracle):
    from oracle import selectors as osel
    g = golden("filtered_selectors")
    for c in g["cases"]:
        B, n, m, M, L, test_mode = [int(x) for x in g[f"{c}__cfg"]]
        kind = str(g[f"{c}__kind"])
        q, beta, tie = g[f"{c}__q"], g[f"{c}__beta"], g[f"{c}__tie_noise"]
        if kind == "sap" or (kind == "egsap" and test_mode):
            gauss = g[f"{c}__gauss_noise"] if f"{c}__gauss_noise" in g else None
            got = osel.filtered_sap(q, beta, M, tie, gauss)
        else:
            got = osel.filtered_greedy(q, beta, M, tie)
        np.testing.assert_array_equal(got, g[f"{c}__actions"], err_msg=str(c))


def test_haal_oracle(golden, oracle):
    from oracle import selectors as osel
    g = golden("haal")
    for c in range(int(g["n_cases"])):
        B, n, m, T, L, N, M, pre, k = [int(x) for x in g[f"h{c}_spec"]]
        for b in range(B):
            a, vals = osel.haal(g[f"h{c}_tables"][b], g[f"h{c}_prios"], g[f"h{c}_T_trans"], float(g[f"h{c}_lambda"]),
                                k, g[f"h{c}_prev"][b], L, T)
            np.testing.assert_array_equal(a, g[f"h{c}_actions"][b])
            np.testing.assert_array_equal(vals, g[f"h{c}_values"][b])
        seqs = osel.time_interval_sequences(min(L, T - k))
        flat = [[t for ti in s for t in ti] for s in seqs]
        assert [list(r[r >= 0]) for r in g[f"h{c}_seqs"]] == flat


def test_haal_variants_oracle(golden, oracle):
    """The HAAL restatement over the power / interference envs (forks carry power states) against
    the reference selector's actions and every sequence's value (tests/golden/haal_variants.npz)."""
    from oracle import selectors as osel
    g = golden("haal_variants")
    for c in range(int(g["n_cases"])):
        kind = str(g[f"h{c}_kind"])
        B, n, m, T, L, N, M, pre, k = [int(x) for x in g[f"h{c}_spec"]]
        for b in range(B):
            a, vals = osel.haal_variant(kind, g[f"h{c}_tables"][b], g[f"h{c}_prios"], np.ones((m, m)) - np.eye(m),
                                        float(g[f"h{c}_lambda"]), k, g[f"h{c}_prev"][b], g[f"h{c}_power"][b], L, T,
                                        bands=g[f"h{c}_bands"], nbr=g[f"h{c}_nbr"])
            np.testing.assert_array_equal(a, g[f"h{c}_actions"][b], err_msg=f"{kind} case {c} env {b}")
            np.testing.assert_array_equal(vals, g[f"h{c}_values"][b], err_msg=f"{kind} case {c} env {b}")
