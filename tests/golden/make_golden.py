"""Generate the golden parity fixtures from the reference implementation.

Runs ONLY in the build container, where the read-only reference checkout lives at
/root/reference. It imports the reference's own Python modules (the reference is
never copied into this repository and never travels to the GPU box) and records
small input/output vectors as .npz files next to this script. Those .npz files are
the pins for both the CPU oracle (oracle/) and the HIP product path.

Offline stand-ins: `gym` is not installed, so a minimal module
providing the names the reference imports is registered in sys.modules; the
orbital-simulator dependencies (astropy, poliastro, h3, shapely) are only needed for
import-time side effects of envs/__init__.py and are satisfied with MagicMock.

Usage:  python tests/golden/make_golden.py          (rewrites every fixture)

Fixture files (all arrays, loaded with numpy.load(allow_pickle=False)):
  mt19937_words.npz   raw legacy-MT19937 32-bit words after np.random.seed(s)
  mock_reset.npz      construct + reset of MockConstellationEnv for several seeds/shapes
  mock_step.npz       per-step rewards / obs / beta / done for injected tables
  lsa.npz             scipy.optimize.linear_sum_assignment input/output pairs
  runner_dumps.npz    EpisodeRunner / ParallelRunner EpisodeBatch dumps (layout + quirks)
  real_env.npz        RealConstellationEnv (injected benefits) reset/step: obs, beta, rewards
  real_variants.npz   RealPowerConstellationEnv / InterferenceConstellationEnv reset/step
  real_bids.npz       the real-env family with bids_as_actions (float32 bids -> scipy LSA) reset/step
  haal_variants.npz   HAALSelector over the power / interference envs (forks carry power states)
  real_runner_dumps.npz  EpisodeRunner + BasicMAC EpisodeBatch dumps over RealConstellationEnv
  filtered_selectors.npz the filtered selectors' actions with their recorded random draws
  haal.npz            HAALSelector actions + every time-interval sequence's value
  replay_buffer.npz   ReplayBuffer ring inserts, counters and seeded samples
  yaml_runner_dumps.npz  EpisodeRunner dumps of the unchanged mock_constellation_iql / _reda
                      configs (20 x 25, agent "rnn", use_rnn False, jumpstart_mac), past both anneals

  python tests/golden/make_golden.py round2   (only the filtered / HAAL / buffer fixtures)
  python tests/golden/make_golden.py yaml     (only yaml_runner_dumps.npz)
"""
import os
import sys
import types
from types import SimpleNamespace
from unittest import mock

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------
# offline stand-ins
# ----------------------------------------------------------------------------------
class _GymEnv:  # the reference only subclasses gym.Env
    pass


class _GymObservationWrapper:
    def __init__(self, env=None):
        self.env = env


class _Space:
    def __init__(self, *a, **k):
        self.args, self.kwargs = a, k


class _Tuple(_Space):
    pass


class _Discrete(_Space):
    pass


class _Box(_Space):
    pass


def _flatdim(space):
    return 0


def _np_random(seed=None):
    # gym's helper builds a private generator; it never touches the global stream
    return np.random.RandomState(), seed


class _TimeLimit:
    def __init__(self, env, max_episode_steps=None):
        self.env = env


def _install_stubs():
    # module-level classes so that envs stay picklable across the ParallelRunner pipes
    gym = types.ModuleType("gym")
    Env, ObservationWrapper = _GymEnv, _GymObservationWrapper
    spaces = types.ModuleType("gym.spaces")
    spaces.Tuple, spaces.Discrete, spaces.Box, spaces.flatdim = _Tuple, _Discrete, _Box, _flatdim
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")
    np_random = _np_random
    seeding.np_random = np_random
    utils.seeding = seeding
    envs_mod = types.ModuleType("gym.envs")
    envs_mod.registry = {}
    wrappers = types.ModuleType("gym.wrappers")
    wrappers.TimeLimit = _TimeLimit
    gym.Env, gym.ObservationWrapper, gym.spaces = Env, ObservationWrapper, spaces
    gym.utils, gym.envs, gym.wrappers = utils, envs_mod, wrappers
    for name, mod in {"gym": gym, "gym.spaces": spaces, "gym.utils": utils,
                      "gym.utils.seeding": seeding, "gym.envs": envs_mod,
                      "gym.wrappers": wrappers}.items():
        sys.modules[name] = mod
    for name in ["astropy", "astropy.units", "poliastro", "poliastro.bodies",
                 "poliastro.twobody", "poliastro.spheroid_location", "poliastro.core",
                 "poliastro.core.events", "h3", "shapely", "shapely.geometry"]:
        sys.modules[name] = mock.MagicMock()
    sys.path.insert(0, REF_SRC)


# ----------------------------------------------------------------------------------
def gen_mt_words():
    seeds = np.array([0, 1, 7, 42, 12345, 2**32 - 1], dtype=np.uint64)
    words = np.stack([np.random.RandomState(int(s)).randint(0, 2**32, size=1400, dtype=np.uint32)
                      for s in seeds])
    # derived draws used by the env (Appendix A): rand / uniform / choice / permutation
    rs = np.random.RandomState(3)
    rand = rs.rand(50)
    rs = np.random.RandomState(3)
    uni = np.array([rs.uniform(0, 20) for _ in range(25)])
    perms = []
    for m in (1, 2, 3, 4, 5, 16, 64, 100, 256):
        rs = np.random.RandomState(m)
        perms.append(np.pad(rs.permutation(m), (0, 256 - m), constant_values=-1))
    np.savez_compressed(os.path.join(OUT, "mt19937_words.npz"), seeds=seeds, words=words,
                        rand_seed3=rand, uniform0_20_seed3=uni,
                        perm_sizes=np.array([1, 2, 3, 4, 5, 16, 64, 100, 256]),
                        perms=np.stack(perms))


def gen_mock_reset():
    from envs.mock_constellation_env import MockConstellationEnv
    cases = [(4, 4, 5, 3, s) for s in (0, 1, 2, 3, 4)] + \
            [(16, 16, 20, 3, s) for s in (0, 1, 7)] + \
            [(8, 12, 6, 4, 5), (3, 10, 4, 6, 11), (64, 64, 20, 3, 0)]
    out = {}
    for idx, (n, m, T, L, s) in enumerate(cases):
        np.random.seed(s)
        env = MockConstellationEnv(n, m, T, L, 0.5)
        init_tab = env.sat_prox_mat.copy()
        env.reset()
        st = np.random.get_state()
        out[f"c{idx}_shape"] = np.array([n, m, T, L, s])
        out[f"c{idx}_init_table"] = init_tab
        out[f"c{idx}_table"] = env.sat_prox_mat
        out[f"c{idx}_prev_assigns"] = np.asarray(env.prev_assigns, dtype=np.int64)
        out[f"c{idx}_obs"] = np.array(env._obs)
        out[f"c{idx}_beta"] = np.asarray(env.beta)
        out[f"c{idx}_mt_key_after"] = st[1]
        out[f"c{idx}_mt_pos_after"] = np.array(st[2])
    out["n_cases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(OUT, "mock_reset.npz"), **out)


def gen_mock_step():
    """Injected tables + fixed action sequences through reset/step."""
    from envs.mock_constellation_env import MockConstellationEnv, generate_benefits_over_time
    rng = np.random.RandomState(1234)
    out = {}
    cases = []
    # (n, m, T, L, lambda, kind)
    specs = [(4, 4, 5, 3, 0.5, "random"), (4, 4, 5, 3, 0.5, "collide"),
             (16, 16, 20, 3, 0.5, "random"), (16, 16, 20, 3, 0.5, "collide"),
             (8, 12, 7, 2, 0.25, "random"), (7, 10, 6, 3, 0.5, "collide"),
             (16, 16, 8, 3, 0.5, "bids"), (6, 6, 5, 2, 0.5, "bids_int"),
             (16, 16, 10, 3, 1.5, "dense"), (5, 9, 4, 5, 0.5, "random")]
    for idx, (n, m, T, L, lam, kind) in enumerate(specs):
        np.random.seed(100 + idx)
        if kind == "dense":
            table = rng.uniform(0.0, 1.0, size=(n, m, T)) + 1e-3
        else:
            table = generate_benefits_over_time(n, m, T, 3, 6)
        # a few exact zeros and tiny values around the 1e-12 mask threshold
        table[0, 0, :] = 0.0
        if n > 1 and m > 1:
            table[1, 1, :] = 1e-13
            table[0, 1, :] = 2e-12
        bids = kind.startswith("bids")
        env = MockConstellationEnv(n, m, T, L, lam, bids_as_actions=bids, sat_prox_mat=table.copy())
        env.reset()
        prev0 = np.asarray(env.prev_assigns, dtype=np.int64)
        obs0 = np.array(env._obs)
        beta0 = np.asarray(env.beta).copy()
        acts, rews, obs, betas, dones, prevs = [], [], [], [], [], []
        for t in range(T):
            if kind == "collide":
                a = np.full(n, t % m, dtype=np.int64) if t % 2 == 0 else rng.randint(0, min(2, m), size=n)
            elif kind == "bids":
                a = rng.uniform(0, 1, size=(n, m)).astype(np.float32)
            elif kind == "bids_int":
                a = rng.randint(0, 3, size=(n, m)).astype(np.float32)
            else:
                a = rng.randint(0, m, size=n)
            r, d, info = env.step(a.copy() if bids else list(a))
            acts.append(np.asarray(a))
            rews.append(np.asarray(r, dtype=np.float64))
            obs.append(np.array(env._obs))
            betas.append(np.asarray(env.beta).copy())
            dones.append(bool(d))
            prevs.append(np.asarray(env.prev_assigns, dtype=np.int64))
        out[f"c{idx}_spec"] = np.array([n, m, T, L])
        out[f"c{idx}_lambda"] = np.array(lam)
        out[f"c{idx}_kind"] = np.array(kind)
        out[f"c{idx}_table"] = table
        out[f"c{idx}_prev0"] = prev0
        out[f"c{idx}_obs0"] = obs0
        out[f"c{idx}_beta0"] = beta0
        out[f"c{idx}_actions"] = np.stack(acts)
        out[f"c{idx}_rewards"] = np.stack(rews)
        out[f"c{idx}_obs"] = np.stack(obs)
        out[f"c{idx}_beta"] = np.stack(betas)
        out[f"c{idx}_done"] = np.array(dones)
        out[f"c{idx}_prev"] = np.stack(prevs)
        cases.append(idx)
    # beta_hat on a time-batched state (HAA call shape) with a custom T_trans
    np.random.seed(9)
    n, m = 6, 7
    T_trans = (rng.uniform(size=(m, m)) > 0.5).astype(np.float64)
    env = MockConstellationEnv(n, m, 4, 2, 0.7, sat_prox_mat=np.ones((n, m, 4)), T_trans=T_trans)
    beta = rng.uniform(-0.2, 1.0, size=(3, n, m))
    beta[beta < 0] = 0.0
    prev = rng.randint(0, m, size=(3, n))
    out["bh_T_trans"] = T_trans
    out["bh_beta"] = beta
    out["bh_prev"] = prev
    out["bh_lambda"] = np.array(0.7)
    out["bh_out"] = env.beta_hat(beta, prev)
    out["bh_out2d"] = env.beta_hat(beta[0], prev[0])
    out["n_cases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(OUT, "mock_step.npz"), **out)


def gen_real_env():
    """RealConstellationEnv (constant-benefit path: injected sat_prox_mat + graphs) through
    reset/step.  Strictly positive tables: no equal totals, so numpy's (unstable) argsort
    order is the tie-free order the GPU restates."""
    from envs.real_constellation_env import RealConstellationEnv
    rng = np.random.RandomState(4321)
    out = {}
    # (n, m, T, L, N, M, lambda, prios, T_trans, actions)
    specs = [(6, 10, 5, 3, 2, 4, 0.5, False, False, "random"),
             (12, 20, 6, 3, 3, 4, 0.5, True, False, "random"),
             (9, 16, 8, 2, 4, 6, 0.3, False, True, "collide"),
             (10, 12, 4, 5, 3, 2, 0.5, True, False, "random"),
             (8, 30, 7, 3, 7, 8, 0.5, False, False, "collide"),
             (5, 9, 6, 3, 4, 6, 1.5, True, True, "random")]
    for idx, (n, m, T, L, N, M, lam, use_prios, use_tt, kind) in enumerate(specs):
        table = rng.uniform(0.01, 1.0, size=(n, m, T))
        prios = rng.uniform(0.5, 2.0, size=m) if use_prios else None
        T_trans = (rng.uniform(size=(m, m)) > 0.4).astype(np.float64) if use_tt else None
        env = RealConstellationEnv(1, n, m, T, N, M, L, lam, sat_prox_mat=table.copy(), graphs=[None] * T,
                                   T_trans=None if T_trans is None else T_trans.copy(),
                                   task_prios=None if prios is None else prios.copy())
        env.reset()
        Le = env.L
        obs0, beta0, prev0 = np.array(env._obs), np.asarray(env.beta).copy(), np.asarray(env.prev_assigns)
        acts, rews, obs, betas, dones, prevs = [], [], [], [], [], []
        for t in range(T):
            if kind == "collide" and t % 2 == 0:
                a = np.full(n, (3 * t) % m, dtype=np.int64)
            else:
                a = rng.randint(0, m, size=n)
            r, d, info = env.step(list(a))
            acts.append(a)
            rews.append(np.asarray(r, dtype=np.float64))
            obs.append(np.array(env._obs))
            betas.append(np.asarray(env.beta).copy())
            dones.append(bool(d))
            prevs.append(np.asarray(env.prev_assigns, dtype=np.int64))
        out[f"r{idx}_spec"] = np.array([n, m, T, Le, N, M])
        out[f"r{idx}_lambda"] = np.array(lam)
        out[f"r{idx}_table"] = table
        out[f"r{idx}_prios"] = prios if prios is not None else np.ones(m)
        out[f"r{idx}_T_trans"] = T_trans if T_trans is not None else np.ones((m, m)) - np.eye(m)
        out[f"r{idx}_obs_size"] = np.array(env.get_obs_size())
        out[f"r{idx}_obs0"] = obs0
        out[f"r{idx}_beta0"] = beta0
        out[f"r{idx}_prev0"] = prev0.astype(np.int64)
        out[f"r{idx}_actions"] = np.stack(acts)
        out[f"r{idx}_rewards"] = np.stack(rews)
        out[f"r{idx}_obs"] = np.stack(obs)
        out[f"r{idx}_beta"] = np.stack(betas)
        out[f"r{idx}_done"] = np.array(dones)
        out[f"r{idx}_prev"] = np.stack(prevs)
    out["n_cases"] = np.array(len(specs))
    np.savez_compressed(os.path.join(OUT, "real_env.npz"), **out)


def gen_real_variants():
    """RealPowerConstellationEnv (injected benefits) and InterferenceConstellationEnv
    (constructed without the orbital simulator: object.__new__ + the attributes its
    __init__ would have derived from it -- sat_prox_mat, neighbor_matrix -- then the
    reference's own reset/step).  Strictly positive tables (tie-free orders); power
    drains over T >= 8 steps so dead agents are exercised."""
    from collections import defaultdict
    from envs.real_power_constellation_env import RealPowerConstellationEnv
    from envs.interference_constellation_env import InterferenceConstellationEnv
    rng = np.random.RandomState(8765)
    out = {}
    specs = [  # (variant, n, m, T, L, N, M, lambda, sparse)
        ("power", 8, 14, 9, 3, 3, 4, 0.5, False), ("power", 10, 16, 10, 2, 4, 6, 0.3, True),
        ("interference", 9, 15, 9, 3, 3, 4, 0.5, False), ("interference", 12, 18, 10, 3, 4, 4, 0.4, True)]
    for idx, (kind, n, m, T, L, N, M, lam, sparse) in enumerate(specs):
        table = rng.uniform(0.01, 1.0, size=(n, m, T))
        if sparse:  # some exact zeros (non-meaningful tasks) without creating equal totals
            table[:, ::5, :] = 0.0
            table[::3, 1::5, :2] = 0.0
        prios = rng.choice([1.0, 1.0, 1.0, 5.0], size=m)
        np.random.seed(500 + idx)
        if kind == "power":
            env = RealPowerConstellationEnv(1, n, m, T, N, M, L, lam, sat_prox_mat=table.copy(), graphs=[None] * T,
                                            task_prios=prios.copy())
            bands = np.zeros(n, dtype=np.int64)
            nbr = np.eye(m, dtype=np.int64)
        else:
            env = object.__new__(InterferenceConstellationEnv)
            env.n, env.m, env.T, env.N, env.M, env.L = n, m, T, N, M, min(L, T)
            env.lambda_, env.beam_types, env.bids_as_actions = lam, 7, False
            env.k, env.done, env.constant_setup = 0, False, True
            env.sat_prox_mat = table.copy()
            nbr = (rng.uniform(size=(m, m)) > 0.7).astype(np.int64)
            nbr = np.maximum(nbr, nbr.T)
            np.fill_diagonal(nbr, 1)
            env.neighbor_matrix = nbr
            bands = rng.randint(0, 3, size=n)
            env.sat_freq_bands = bands
            env.sat_freq_band_dict = defaultdict(list)
            for i, b in enumerate(bands):
                env.sat_freq_band_dict[b].append(i)
            env.task_prios = np.repeat(np.tile(prios, (n, 1))[:, :, np.newaxis], env.L, axis=-1)
            env.power_states = np.ones(n)
        env.reset()
        Le = env.L
        obs0, beta0 = np.array(env._obs), np.asarray(env.beta).copy()
        prev0 = np.asarray(env.prev_assigns, dtype=np.int64).copy()
        acts, rews, obs, betas, dones, prevs, powers = [], [], [], [], [], [], []
        for t in range(T):
            if t % 3 == 1:  # crowd a few tasks: collisions and (for interference) neighbours
                a = rng.randint(0, min(3, m), size=n)
            else:
                a = rng.randint(0, m, size=n)
            r, d, info = env.step(list(a))
            acts.append(a)
            rews.append(np.asarray(r, dtype=np.float64))
            obs.append(np.array(env._obs))
            betas.append(np.asarray(env.beta).copy())
            dones.append(bool(d))
            prevs.append(np.asarray(env.prev_assigns, dtype=np.int64))
            powers.append(np.asarray(env.power_states, dtype=np.float64).copy())
        out[f"v{idx}_kind"] = np.array(kind)
        out[f"v{idx}_spec"] = np.array([n, m, T, Le, N, M])
        out[f"v{idx}_lambda"] = np.array(lam)
        out[f"v{idx}_table"] = table
        out[f"v{idx}_prios"] = prios
        out[f"v{idx}_bands"] = np.asarray(bands, dtype=np.int64)
        out[f"v{idx}_nbr"] = np.asarray(nbr, dtype=np.float64)
        out[f"v{idx}_obs_size"] = np.array(env.get_obs_size())
        out[f"v{idx}_obs0"] = obs0
        out[f"v{idx}_beta0"] = beta0
        out[f"v{idx}_prev0"] = prev0
        out[f"v{idx}_actions"] = np.stack(acts)
        out[f"v{idx}_rewards"] = np.stack(rews)
        out[f"v{idx}_obs"] = np.stack(obs)
        out[f"v{idx}_beta"] = np.stack(betas)
        out[f"v{idx}_done"] = np.array(dones)
        out[f"v{idx}_prev"] = np.stack(prevs)
        out[f"v{idx}_power"] = np.stack(powers)
    out["n_cases"] = np.array(len(specs))
    np.savez_compressed(os.path.join(OUT, "real_variants.npz"), **out)


def gen_real_bids():
    """bids_as_actions on the real-env family (VERDICT r5 "Next" item 4): RealConstellationEnv,
    RealPowerConstellationEnv and InterferenceConstellationEnv constructed with bids_as_actions
    (the latter without the orbital simulator, as gen_real_variants), stepped with float32 bid
    matrices -- the batch's float32 actions row -- so each step is scipy's
    linear_sum_assignment(bids, maximize=True) (real_constellation_env.py:140-142,
    real_power_constellation_env.py:142, interference_constellation_env.py:159).  Continuous
    random bids (tie-free LSA) and strictly positive tables (tie-free argsort orders)."""
    from collections import defaultdict
    from envs.real_constellation_env import RealConstellationEnv
    from envs.real_power_constellation_env import RealPowerConstellationEnv
    from envs.interference_constellation_env import InterferenceConstellationEnv
    rng = np.random.RandomState(2468)
    out = {}
    specs = [  # (variant, n, m, T, L, N, M, lambda)
        ("real", 7, 12, 6, 3, 2, 4, 0.5), ("real", 12, 20, 5, 2, 3, 4, 0.3),
        ("power", 8, 14, 9, 3, 3, 4, 0.5), ("interference", 9, 15, 8, 3, 3, 4, 0.4)]
    for idx, (kind, n, m, T, L, N, M, lam) in enumerate(specs):
        table = rng.uniform(0.01, 1.0, size=(n, m, T))
        prios = rng.choice([1.0, 1.0, 1.0, 5.0], size=m) if kind != "real" else np.ones(m)
        np.random.seed(700 + idx)
        bands = np.zeros(n, dtype=np.int64)
        nbr = np.eye(m, dtype=np.int64)
        if kind == "real":
            env = RealConstellationEnv(1, n, m, T, N, M, L, lam, sat_prox_mat=table.copy(), graphs=[None] * T,
                                       bids_as_actions=True)
        elif kind == "power":
            env = RealPowerConstellationEnv(1, n, m, T, N, M, L, lam, sat_prox_mat=table.copy(), graphs=[None] * T,
                                            task_prios=prios.copy(), bids_as_actions=True)
        else:
            env = object.__new__(InterferenceConstellationEnv)
            env.n, env.m, env.T, env.N, env.M, env.L = n, m, T, N, M, min(L, T)
            env.lambda_, env.beam_types, env.bids_as_actions = lam, 7, True
            env.k, env.done, env.constant_setup = 0, False, True
            env.sat_prox_mat = table.copy()
            nbr = (rng.uniform(size=(m, m)) > 0.7).astype(np.int64)
            nbr = np.maximum(nbr, nbr.T)
            np.fill_diagonal(nbr, 1)
            env.neighbor_matrix = nbr
            bands = rng.randint(0, 3, size=n)
            env.sat_freq_bands = bands
            env.sat_freq_band_dict = defaultdict(list)
            for i, b in enumerate(bands):
                env.sat_freq_band_dict[b].append(i)
            env.task_prios = np.repeat(np.tile(prios, (n, 1))[:, :, np.newaxis], env.L, axis=-1)
            env.power_states = np.ones(n)
        env.reset()
        obs0, beta0 = np.array(env._obs), np.asarray(env.beta).copy()
        prev0 = np.asarray(env.prev_assigns, dtype=np.int64).copy()
        bids_l, rews, obs, betas, dones, prevs, powers = [], [], [], [], [], [], []
        for t in range(T):
            bids = rng.uniform(0.0, 1.0, size=(n, m)).astype(np.float32)
            if t % 3 == 1:  # a few columns everyone wants: contested LSA rows
                bids[:, :2] += 1.0
            r, d, info = env.step(bids)
            bids_l.append(bids)
            rews.append(np.asarray(r, dtype=np.float64))
            obs.append(np.array(env._obs))
            betas.append(np.asarray(env.beta).copy())
            dones.append(bool(d))
            prevs.append(np.asarray(env.prev_assigns, dtype=np.int64))
            powers.append(np.asarray(getattr(env, "power_states", np.ones(n)), dtype=np.float64).copy())
        out[f"b{idx}_kind"] = np.array(kind)
        out[f"b{idx}_spec"] = np.array([n, m, T, env.L, N, M])
        out[f"b{idx}_lambda"] = np.array(lam)
        out[f"b{idx}_table"] = table
        out[f"b{idx}_prios"] = prios
        out[f"b{idx}_bands"] = np.asarray(bands, dtype=np.int64)
        out[f"b{idx}_nbr"] = np.asarray(nbr, dtype=np.float64)
        out[f"b{idx}_obs_size"] = np.array(env.get_obs_size())
        out[f"b{idx}_obs0"] = obs0
        out[f"b{idx}_beta0"] = beta0
        out[f"b{idx}_prev0"] = prev0
        out[f"b{idx}_bids"] = np.stack(bids_l)
        out[f"b{idx}_rewards"] = np.stack(rews)
        out[f"b{idx}_obs"] = np.stack(obs)
        out[f"b{idx}_beta"] = np.stack(betas)
        out[f"b{idx}_done"] = np.array(dones)
        out[f"b{idx}_prev"] = np.stack(prevs)
        out[f"b{idx}_power"] = np.stack(powers)
    out["n_cases"] = np.array(len(specs))
    np.savez_compressed(os.path.join(OUT, "real_bids.npz"), **out)


def gen_lsa():
    import scipy.optimize as so
    rng = np.random.RandomState(77)
    out = {}
    k = 0
    shapes = [(1, 1), (1, 5), (5, 1), (2, 3), (3, 2), (4, 4), (5, 8), (8, 5), (16, 16),
              (7, 7), (10, 13), (13, 10), (64, 64), (33, 64), (64, 40), (100, 100), (3, 0)]
    for (nr, nc) in shapes:
        for kind in ("uniform", "int3", "round1", "const", "neg"):
            for maximize in (False, True):
                if kind == "uniform":
                    C = rng.uniform(-1, 1, size=(nr, nc))
                elif kind == "int3":
                    C = rng.randint(0, 3, size=(nr, nc)).astype(np.float64)
                elif kind == "round1":
                    C = np.round(rng.uniform(0, 1, size=(nr, nc)), 1)
                elif kind == "const":
                    C = np.full((nr, nc), 2.5)
                else:
                    C = -np.exp(rng.normal(size=(nr, nc)) * 3)
                r, c = so.linear_sum_assignment(C, maximize=maximize)
                out[f"k{k}_C"] = C
                out[f"k{k}_max"] = np.array(maximize)
                out[f"k{k}_row"] = r.astype(np.int64)
                out[f"k{k}_col"] = c.astype(np.int64)
                k += 1
    # float32 Q-value-like matrices (the SAP selector casts f32 -> f64)
    for _ in range(20):
        C = rng.normal(size=(16, 16)).astype(np.float32).astype(np.float64)
        r, c = so.linear_sum_assignment(C, maximize=True)
        out[f"k{k}_C"], out[f"k{k}_max"] = C, np.array(True)
        out[f"k{k}_row"], out[f"k{k}_col"] = r.astype(np.int64), c.astype(np.int64)
        k += 1
    # error cases: (C, maximize, expected message fragment)
    errs = []
    bad = np.ones((3, 3)); bad[1, 1] = np.nan
    errs.append((bad, False))
    bad2 = np.ones((3, 3)); bad2[0, 2] = -np.inf
    errs.append((bad2, False))
    bad3 = np.ones((3, 3)); bad3[0, 2] = np.inf
    errs.append((bad3, True))  # +inf under maximize becomes -inf -> invalid
    inf = np.full((3, 3), np.inf); inf[0, 0] = 1.0; inf[1, 0] = 1.0
    errs.append((inf, False))  # infeasible
    for i, (C, mx) in enumerate(errs):
        try:
            so.linear_sum_assignment(C, maximize=mx)
            msg = "ok"
        except ValueError as e:
            msg = str(e)
        out[f"e{i}_C"], out[f"e{i}_max"], out[f"e{i}_msg"] = C, np.array(mx), np.array(msg)
    out["n_cases"], out["n_err"] = np.array(k), np.array(len(errs))
    np.savez_compressed(os.path.join(OUT, "lsa.npz"), **out)


class _Logger:
    def __init__(self):
        self.stats = []

    def log_stat(self, k, v, t):
        self.stats.append((k, float(v), int(t)))


def _args(**kw):
    base = dict(batch_size_run=1, env="mock_constellation_env",
                env_args=dict(n=4, m=4, T=5, L=3, lambda_=0.5, bids_as_actions=False, seed=0),
                use_mps_action_selection=False, mac="basic_mac", test_nepisode=1,
                runner_log_interval=10**9, render=False, agent="rnn", hidden_dim=64, use_rnn=True,
                obs_last_action=False, obs_agent_id=False, agent_output_type="q",
                action_selector="epsilon_greedy", epsilon_start=0.0, epsilon_finish=0.0,
                epsilon_anneal_time=1000, evaluation_epsilon=0.0, device="cpu",
                jumpstart_action_selector="haa_selector", jumpstart_epsilon_start=1.0,
                jumpstart_epsilon_finish=1.0, jumpstart_epsilon_anneal_time=1000,
                jumpstart_evaluation_epsilon=1.0)
    base.update(kw)
    return SimpleNamespace(**base)


def gen_runner_dumps():
    import torch as th
    th.set_num_threads(1)
    from runners.episode_runner import EpisodeRunner
    from runners.parallel_runner import ParallelRunner
    from controllers import REGISTRY as mac_REGISTRY

    out = {}
    runs = [  # (tag, runner, n, m, T, B, selector, mac, use_rnn)
        ("ep_eg_4", "episode", 4, 4, 5, 1, "epsilon_greedy", "basic_mac", True),
        ("ep_sap_8", "episode", 8, 8, 6, 1, "sap", "basic_mac", False),
        ("par_eg_6", "parallel", 6, 6, 5, 3, "epsilon_greedy", "basic_mac", True),
        ("par_sap_8", "parallel", 8, 8, 6, 3, "sap", "basic_mac", True),
        ("ep_haa_8", "episode", 8, 8, 6, 1, "sap", "jumpstart_mac", False),
    ]
    for ri, (tag, rname, n, m, T, B, sel, macname, use_rnn) in enumerate(runs):
        seed = 10 + ri
        np.random.seed(seed)
        th.manual_seed(seed)
        args = _args(batch_size_run=B, mac=macname, action_selector=sel, use_rnn=use_rnn,
                     env_args=dict(n=n, m=m, T=T, L=3, lambda_=0.5, bids_as_actions=False, seed=seed))
        logger = _Logger()
        runner = (EpisodeRunner if rname == "episode" else ParallelRunner)(args, logger)
        env = runner.get_env()
        args.n, args.m, args.T = env.n, env.m, env.T
        groups = {"agents": n}
        mac = mac_REGISTRY[macname](env.scheme, groups, args)
        # deterministic, non-trivial weights shared by the training and selector copies
        g = th.Generator().manual_seed(1000 + ri)
        with th.no_grad():
            for p in mac.agent.parameters():
                p.copy_(th.randn(p.shape, generator=g) * 0.3)
        mac.update_action_selector_agent()
        runner.setup(scheme=env.scheme, groups=groups, preprocess=env.preprocess, mac=mac)
        batch = runner.run(test_mode=False)
        for k, v in batch.data.transition_data.items():
            out[f"{tag}__{k}"] = v.numpy()
        sd = mac.agent.state_dict()
        for k, v in sd.items():
            out[f"{tag}__w__{k}"] = v.numpy()
        out[f"{tag}__returns"] = np.asarray(runner.train_returns, dtype=np.float64)
        out[f"{tag}__t_env"] = np.array(runner.t_env)
        out[f"{tag}__cfg"] = np.array([n, m, T, B, seed, int(use_rnn)])
        out[f"{tag}__names"] = np.array([rname, sel, macname])
        if rname == "parallel":
            runner.close_env()
    np.savez_compressed(os.path.join(OUT, "runner_dumps.npz"), **out)


def _ref_yaml_config(alg):
    """default.yaml <- envs/mock_constellation_env.yaml <- algs/<alg>.yaml, merged as the
    reference's main.py:59-65 / 92-104 merges them (read as data with yaml.safe_load)."""
    import yaml

    def load(rel):
        with open(os.path.join(REF_SRC, "config", rel)) as f:
            return yaml.safe_load(f)

    def merge(d, u):
        for k, v in u.items():
            d[k] = merge(dict(d.get(k) or {}), v) if isinstance(v, dict) else v
        return d

    cfg = load("default.yaml")
    merge(cfg, load("envs/mock_constellation_env.yaml"))
    merge(cfg, load(f"algs/{alg}.yaml"))
    return cfg


def gen_yaml_runner_dumps():
    """EpisodeRunner dumps of the reference's UNCHANGED mock algorithm configs
    (mock_constellation_iql.yaml / mock_constellation_reda.yaml on
    envs/mock_constellation_env.yaml: 20 agents x 25 tasks, T 20, L 3, agent "rnn", use_rnn
    False, jumpstart_mac with the HAA jumpstart selector).  runner.t_env starts at 20,000, past
    both epsilon anneals (1 -> 0 over 20,000 env steps): the jumpstart coin never picks HAA and
    the RL selector is greedy (epsilon-greedy) / noise-free (SAP), so the episode is
    deterministic given the seed and the agent weights recorded here."""
    import torch as th
    th.set_num_threads(1)
    from runners.episode_runner import EpisodeRunner
    from controllers import REGISTRY as mac_REGISTRY

    out = {}
    for ri, (tag, alg) in enumerate([("iql", "mock_constellation_iql"), ("reda", "mock_constellation_reda")]):
        cfg = _ref_yaml_config(alg)
        seed = 40 + ri
        cfg["env_args"] = dict(cfg["env_args"], seed=seed)
        cfg.update(batch_size_run=1, device="cpu", use_cuda=False, seed=seed, runner="episode")
        args = SimpleNamespace(**cfg)
        np.random.seed(seed)
        th.manual_seed(seed)
        logger = _Logger()
        runner = EpisodeRunner(args, logger)
        env = runner.get_env()
        args.n, args.m, args.T = env.n, env.m, env.T
        groups = {"agents": env.n}
        mac = mac_REGISTRY[args.mac](env.scheme, groups, args)
        g = th.Generator().manual_seed(2000 + ri)
        with th.no_grad():
            for p in mac.agent.parameters():
                p.copy_(th.randn(p.shape, generator=g) * 0.3)
        mac.update_action_selector_agent()
        runner.setup(scheme=env.scheme, groups=groups, preprocess=env.preprocess, mac=mac)
        runner.t_env = 20000
        batch = runner.run(test_mode=False)
        for k, v in batch.data.transition_data.items():
            out[f"{tag}__{k}"] = v.numpy()
        for k, v in mac.agent.state_dict().items():
            out[f"{tag}__w__{k}"] = v.numpy()
        # the runner logged (and cleared) its returns at this t_env: one env, so return_mean is it
        rets = [v for k, v, t in logger.stats if k == "return_mean"] or list(runner.train_returns)
        out[f"{tag}__returns"] = np.asarray(rets, dtype=np.float64)
        out[f"{tag}__t_env"] = np.array(runner.t_env)
        out[f"{tag}__cfg"] = np.array([env.n, env.m, env.T, int(args.env_args["L"]), seed, int(bool(args.use_rnn)),
                                       20000])
        out[f"{tag}__lambda"] = np.array(float(args.env_args["lambda_"]))
        out[f"{tag}__names"] = np.array([args.mac, args.action_selector, args.agent, args.jumpstart_action_selector])
        out[f"{tag}__sched"] = np.array([args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                         args.jumpstart_epsilon_start, args.jumpstart_epsilon_finish,
                                         args.jumpstart_epsilon_anneal_time], dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "yaml_runner_dumps.npz"), **out)


def gen_real_runner_dumps():
    """EpisodeRunner + BasicMAC over RealConstellationEnv (constant benefits injected
    through env_args: sat_prox_mat + graphs), greedy epsilon-greedy and SAP selectors.
    Strictly positive tables, so the env's argsorts are tie-free."""
    import torch as th
    th.set_num_threads(1)
    from runners.episode_runner import EpisodeRunner
    from controllers import REGISTRY as mac_REGISTRY

    out = {}
    runs = [  # (tag, n, m, T, N, M, L, lambda, selector, use_rnn, prios)
        ("real_eg_16", 12, 16, 6, 3, 4, 3, 0.5, "epsilon_greedy", True, False),
        ("real_sap_16", 10, 16, 5, 2, 4, 2, 0.5, "sap", True, True),
        ("real_eg_32", 20, 32, 5, 4, 6, 3, 0.3, "epsilon_greedy", False, True),
    ]
    for ri, (tag, n, m, T, N, M, L, lam, sel, use_rnn, use_prios) in enumerate(runs):
        seed = 40 + ri
        rng = np.random.RandomState(seed)
        table = rng.uniform(0.01, 1.0, size=(n, m, T))
        prios = rng.uniform(0.5, 2.0, size=m) if use_prios else None
        np.random.seed(seed)
        th.manual_seed(seed)
        env_args = dict(num_planes=1, num_sats_per_plane=n, m=m, T=T, N=N, M=M, L=L, lambda_=lam,
                        sat_prox_mat=table.copy(), graphs=[None] * T,
                        task_prios=None if prios is None else prios.copy())
        args = _args(env="real_constellation_env", env_args=env_args, action_selector=sel, use_rnn=use_rnn)
        runner = EpisodeRunner(args, _Logger())
        env = runner.get_env()
        args.n, args.m, args.T = env.n, env.m, env.T
        mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
        g = th.Generator().manual_seed(2000 + ri)
        with th.no_grad():
            for p in mac.agent.parameters():
                p.copy_(th.randn(p.shape, generator=g) * 0.3)
        mac.update_action_selector_agent()
        runner.setup(scheme=env.scheme, groups={"agents": n}, preprocess=env.preprocess, mac=mac)
        batch = runner.run(test_mode=False)
        for k, v in batch.data.transition_data.items():
            out[f"{tag}__{k}"] = v.numpy()
        for k, v in mac.agent.state_dict().items():
            out[f"{tag}__w__{k}"] = v.numpy()
        out[f"{tag}__returns"] = np.asarray(runner.train_returns, dtype=np.float64)
        out[f"{tag}__t_env"] = np.array(runner.t_env)
        out[f"{tag}__cfg"] = np.array([n, m, T, N, M, L, int(use_rnn)])
        out[f"{tag}__lambda"] = np.array(lam)
        out[f"{tag}__table"] = table
        out[f"{tag}__prios"] = prios if prios is not None else np.ones(m)
        out[f"{tag}__names"] = np.array([sel])
    np.savez_compressed(os.path.join(OUT, "real_runner_dumps.npz"), **out)


def _f16_topm_tiefree(rng, n, m, L, M, zero_frac):
    """float16 beta [n, m, L] whose float16 L-sums (torch's Half sum) have M + 1 distinct
    leading values per agent, so torch.topk's unspecified tie order cannot matter; a
    `zero_frac` share of each agent's other tasks is all-zero (the real env's invisible
    tasks, which tie at 0 below the top M)."""
    import torch as th
    beta = np.zeros((n, m, L), dtype=np.float16)
    for i in range(n):
        while True:
            row = rng.uniform(0.0, 1.5, size=(m, L)).astype(np.float16)
            zero = rng.uniform(size=m) < zero_frac
            zero[rng.choice(m, M + 1, replace=False)] = False
            row[zero] = 0
            tot = th.from_numpy(row).sum(-1).numpy().astype(np.float64)
            top = np.sort(tot)[::-1][:M + 1]
            if np.all(np.diff(top) < 0):
                beta[i] = row
                break
    return beta


def gen_filtered_selectors():
    """FilteredSAPActionSelector / FilteredEpsGrSAPTestActionSelector
    (filtered_sap_selectors.py:7-148) and FilteredEpsilonGreedyActionSelector
    (filtered_classic_selectors.py:6-67) called on seeded Q-values [B, n, M+1] and float16
    beta [B, n, m, L].  Every torch.rand_like / torch.normal draw the selectors make is
    recorded (the 1e-8 tie-breaking noise, the Gaussian exploration noise), so the GPU
    selectors can be fed the same draws and compared bit for bit.  The top-M boundary of
    every row is tie-free (torch.topk leaves tie order unspecified)."""
    import torch as th
    th.set_num_threads(1)
    import action_selectors.filtered_sap_selectors as fsap
    import action_selectors.filtered_classic_selectors as fcls

    rec = {"rand_like": [], "normal": []}
    real_rand_like, real_normal = th.rand_like, th.normal

    def rand_like(*a, **k):
        r = real_rand_like(*a, **k)
        rec["rand_like"].append(r.clone())
        return r

    def normal(*a, **k):
        r = real_normal(*a, **k)
        rec["normal"].append(r.clone())
        return r

    out = {}
    rng = np.random.RandomState(777)
    # (tag, selector class, B, n, m, M, L, epsilon, test_mode, q scale, zero_frac)
    cases = [("sap_e0", "sap", 3, 10, 24, 4, 3, 0.0, False, 1.0, 0.5),
             ("sap_e03", "sap", 3, 12, 30, 6, 3, 0.3, False, 1.0, 0.3),
             ("sap_small_q", "sap", 2, 9, 20, 4, 2, 0.0, False, 1e-3, 0.6),
             ("sap_eval", "sap", 2, 8, 16, 4, 3, 0.7, True, 1.0, 0.0),
             ("egsap_test", "egsap", 3, 10, 24, 4, 3, 0.5, True, 1.0, 0.5),
             ("egsap_train_e0", "egsap", 3, 10, 24, 4, 3, 0.0, False, 1e-2, 0.5),
             ("eg_e0", "eg", 4, 12, 40, 6, 3, 0.0, False, 1.0, 0.4),
             ("eg_eval", "eg", 2, 7, 18, 5, 2, 0.9, True, 1e-3, 0.0),
             ("sap_big", "sap", 2, 36, 60, 10, 3, 0.0, False, 1.0, 0.7)]
    with mock.patch.object(th, "rand_like", rand_like), mock.patch.object(th, "normal", normal):
        for tag, kind, B, n, m, M, L, eps, test_mode, qs, zf in cases:
            q = (rng.standard_normal((B, n, M + 1)) * qs).astype(np.float32)
            # the baseline (column M) near the other values: exact float32 ties among the
            # "do nothing" columns where the 1e-8 noise rounds away
            beta = np.stack([_f16_topm_tiefree(rng, n, m, L, M, zf) for _ in range(B)])
            avail = np.ones((B, n, m), dtype=np.int64)
            args = SimpleNamespace(epsilon_start=eps, epsilon_finish=eps, epsilon_anneal_time=1000,
                                   evaluation_epsilon=0.0, use_mps_action_selection=False, device="cpu",
                                   env_args={"M": M})
            cls = {"sap": fsap.FilteredSAPActionSelector, "egsap": fsap.FilteredEpsGrSAPTestActionSelector,
                   "eg": fcls.FilteredEpsilonGreedyActionSelector}[kind]
            sel = cls(args)
            rec["rand_like"].clear()
            rec["normal"].clear()
            th.manual_seed(1234)
            acts = sel.select_action(th.from_numpy(q), th.from_numpy(avail), 0, test_mode=test_mode,
                                     beta=th.from_numpy(beta))
            out[f"{tag}__q"] = q
            out[f"{tag}__beta"] = beta
            out[f"{tag}__cfg"] = np.array([B, n, m, M, L, int(test_mode)])
            out[f"{tag}__kind"] = np.array(kind)
            out[f"{tag}__epsilon"] = np.array(eps)
            out[f"{tag}__actions"] = acts.numpy()
            out[f"{tag}__actions_dtype"] = np.array(str(acts.dtype))
            # tie noise: one [n, m] draw per env (the SAP loops) or one [B, n, m] draw
            tie = [r.numpy() for r in rec["rand_like"] if r.dim() >= 2 and r.shape[-1] == m]
            out[f"{tag}__tie_noise"] = np.stack(tie).reshape(B, n, m)
            gauss = [r.numpy() for r in rec["normal"]]
            if gauss:
                out[f"{tag}__gauss_noise"] = np.stack(gauss).reshape(B, n, m)
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(OUT, "filtered_selectors.npz"), **out)


def gen_haal():
    """HAALSelector (non_rl_selectors.py:54-118) over RealConstellationEnv (injected
    benefits): the reference's own selector on deep-copied envs at several steps, plus the
    value of every time-interval sequence computed by the same deepcopy + step loop (the
    selector discards them; the GPU form reports them)."""
    import copy
    import torch as th
    from envs.real_constellation_env import RealConstellationEnv
    from action_selectors.non_rl_selectors import HAALSelector
    from utils.methods import generate_all_time_intervals, build_time_interval_sequences
    import scipy.optimize as so
    rng = np.random.RandomState(99)
    out = {}
    # (n, m, T, L, N, M, lambda, prios, T_trans, steps before the selection)
    specs = [(6, 10, 5, 3, 2, 4, 0.5, False, False, 0),
             (8, 14, 6, 3, 2, 4, 0.5, True, False, 2),
             (7, 12, 6, 4, 2, 4, 0.3, False, True, 1),
             (5, 9, 5, 3, 2, 4, 1.5, True, False, 3),
             (9, 16, 7, 2, 3, 6, 0.5, False, False, 4)]
    for idx, (n, m, T, L, N, M, lam, use_prios, use_tt, pre) in enumerate(specs):
        B = 3
        envs, tables, prev_l = [], [], []
        prios = rng.uniform(0.5, 2.0, size=m) if use_prios else None
        T_trans = (rng.uniform(size=(m, m)) > 0.4).astype(np.float64) if use_tt else None
        for b in range(B):
            table = rng.uniform(0.01, 1.0, size=(n, m, T))
            table[rng.uniform(size=table.shape) < 0.3] = 0.0  # invisible pairs: beta_hat mask
            env = RealConstellationEnv(1, n, m, T, N, M, L, lam, sat_prox_mat=table.copy(), graphs=[None] * T,
                                       T_trans=None if T_trans is None else T_trans.copy(),
                                       task_prios=None if prios is None else prios.copy())
            env.reset()
            for t in range(pre):
                env.step(list(rng.randint(0, m, size=n)))
            envs.append(env)
            tables.append(table)
            prev_l.append(np.asarray(env.prev_assigns, dtype=np.int64))
        args = SimpleNamespace(runner="episode", use_mps_action_selection=False, device="cpu")
        sel = HAALSelector(args)
        sel.envs = envs
        scheme = {"beta": {"vshape": (n, m, L), "part_of_state": True},
                  "prev_assigns": {"vshape": (n,), "part_of_state": True}}
        batch = SimpleNamespace(scheme=scheme)
        beta5 = th.zeros((B, 1, n, m, envs[0].L))
        batch_get = {"beta": beta5}
        batch = type("B", (), {"scheme": scheme, "__getitem__": lambda self, k: batch_get[k]})()
        acts = sel.select_action(batch).numpy()
        # the discarded per-sequence values: the selector's own loop, recorded
        eff = min(envs[0].L, envs[0].T - envs[0].k)
        seqs = build_time_interval_sequences(generate_all_time_intervals(eff), eff)
        vals = np.zeros((B, len(seqs)))
        for b in range(B):
            for s, tis in enumerate(seqs):
                e = copy.deepcopy(envs[b])
                tot = 0
                for ti in tis:
                    bh = e.beta_hat(e.beta, e.prev_assigns)
                    _, a = so.linear_sum_assignment(bh.sum(axis=-1), maximize=True)
                    for _ in range(ti[1] - ti[0] + 1):
                        r, _, _ = e.step(a)
                        tot += sum(r)
                vals[b, s] = tot
        out[f"h{idx}_spec"] = np.array([B, n, m, T, envs[0].L, N, M, pre, envs[0].k])
        out[f"h{idx}_lambda"] = np.array(lam)
        out[f"h{idx}_tables"] = np.stack(tables)
        out[f"h{idx}_prios"] = prios if prios is not None else np.ones(m)
        out[f"h{idx}_T_trans"] = T_trans if T_trans is not None else np.ones((m, m)) - np.eye(m)
        out[f"h{idx}_prev"] = np.stack(prev_l)
        out[f"h{idx}_actions"] = acts
        out[f"h{idx}_values"] = vals
        out[f"h{idx}_seqs"] = np.array([[t for ti in tis for t in ti] + [-1] * (2 * eff - 2 * len(tis))
                                        for tis in seqs])
    out["n_cases"] = np.array(len(specs))
    np.savez_compressed(os.path.join(OUT, "haal.npz"), **out)


def gen_haal_variants():
    """HAALSelector (non_rl_selectors.py:54-118) over RealPowerConstellationEnv and
    InterferenceConstellationEnv (VERDICT r5 "Next" item 8): the selector deep-copies the env --
    power states included -- and steps the copies, so forks drain / recharge power
    (real_power_constellation_env.py:170-178) and see power-zeroed beta_hat rows (:343-347).
    The reference's own selector after `pre` steps (some satellites dead or below 1e-12 power),
    plus every sequence's value by the selector's own deepcopy + get_state + step loop."""
    import copy
    from collections import defaultdict
    import torch as th
    from envs.real_power_constellation_env import RealPowerConstellationEnv
    from envs.interference_constellation_env import InterferenceConstellationEnv
    from action_selectors.non_rl_selectors import HAALSelector
    from utils.methods import generate_all_time_intervals, build_time_interval_sequences
    import scipy.optimize as so
    rng = np.random.RandomState(1357)
    out = {}
    # (variant, n, m, T, L, N, M, lambda, steps before the selection)
    specs = [("power", 7, 12, 10, 3, 2, 4, 0.5, 5), ("power", 8, 14, 10, 4, 2, 4, 0.3, 4),
             ("power", 6, 10, 9, 3, 2, 4, 0.5, 0), ("interference", 8, 13, 9, 3, 2, 4, 0.4, 5),
             ("interference", 9, 15, 8, 4, 3, 4, 0.5, 2)]
    for idx, (kind, n, m, T, L, N, M, lam, pre) in enumerate(specs):
        B = 3
        prios = rng.choice([1.0, 1.0, 1.0, 5.0], size=m)
        nbr = (rng.uniform(size=(m, m)) > 0.7).astype(np.int64)
        nbr = np.maximum(nbr, nbr.T)
        np.fill_diagonal(nbr, 1)
        bands = rng.randint(0, 3, size=n)
        envs, tables, prev0_l, prev_l, power_l, acts_pre = [], [], [], [], [], []
        for b in range(B):
            table = rng.uniform(0.01, 1.0, size=(n, m, T))
            table[rng.uniform(size=table.shape) < 0.3] = 0.0  # invisible pairs: no drain, no penalty
            np.random.seed(900 + 10 * idx + b)
            if kind == "power":
                env = RealPowerConstellationEnv(1, n, m, T, N, M, L, lam, sat_prox_mat=table.copy(),
                                                graphs=[None] * T, task_prios=prios.copy())
            else:
                env = object.__new__(InterferenceConstellationEnv)
                env.n, env.m, env.T, env.N, env.M, env.L = n, m, T, N, M, min(L, T)
                env.lambda_, env.beam_types, env.bids_as_actions = lam, 7, False
                env.k, env.done, env.constant_setup = 0, False, True
                env.sat_prox_mat = table.copy()
                env.neighbor_matrix = nbr
                env.sat_freq_bands = bands
                env.sat_freq_band_dict = defaultdict(list)
                for i, bd in enumerate(bands):
                    env.sat_freq_band_dict[bd].append(i)
                env.task_prios = np.repeat(np.tile(prios, (n, 1))[:, :, np.newaxis], env.L, axis=-1)
                env.power_states = np.ones(n)
            env.reset()
            prev0_l.append(np.asarray(env.prev_assigns, dtype=np.int64).copy())
            ap = []
            for t in range(pre):
                a = rng.randint(0, m, size=n)
                env.step(list(a))
                ap.append(a)
            envs.append(env)
            tables.append(table)
            prev_l.append(np.asarray(env.prev_assigns, dtype=np.int64))
            power_l.append(np.asarray(env.power_states, dtype=np.float64).copy())
            acts_pre.append(np.stack(ap) if pre else np.zeros((0, n), np.int64))
        args = SimpleNamespace(runner="episode", use_mps_action_selection=False, device="cpu")
        sel = HAALSelector(args)
        sel.envs = envs
        scheme = {"beta": {"vshape": (n, m, L), "part_of_state": True},
                  "prev_assigns": {"vshape": (n,), "part_of_state": True},
                  "power_states": {"vshape": (n,), "part_of_state": True}}
        beta5 = th.zeros((B, 1, n, m, envs[0].L))
        batch_get = {"beta": beta5}
        batch = type("B", (), {"scheme": scheme, "__getitem__": lambda self, k: batch_get[k]})()
        acts = sel.select_action(batch).numpy()
        eff = min(envs[0].L, envs[0].T - envs[0].k)
        seqs = build_time_interval_sequences(generate_all_time_intervals(eff), eff)
        vals = np.zeros((B, len(seqs)))
        for b in range(B):
            for s_, tis in enumerate(seqs):
                e = copy.deepcopy(envs[b])
                tot = 0
                for ti in tis:
                    bh = e.beta_hat(e.beta, e.prev_assigns, e.power_states)
                    _, a = so.linear_sum_assignment(bh.sum(axis=-1), maximize=True)
                    for _ in range(ti[1] - ti[0] + 1):
                        r, _, _ = e.step(a)
                        tot += sum(r)
                vals[b, s_] = tot
        out[f"h{idx}_kind"] = np.array(kind)
        out[f"h{idx}_spec"] = np.array([B, n, m, T, envs[0].L, N, M, pre, envs[0].k])
        out[f"h{idx}_lambda"] = np.array(lam)
        out[f"h{idx}_tables"] = np.stack(tables)
        out[f"h{idx}_prios"] = prios
        out[f"h{idx}_bands"] = np.asarray(bands, dtype=np.int64)
        out[f"h{idx}_nbr"] = np.asarray(nbr, dtype=np.float64)
        out[f"h{idx}_prev0"] = np.stack(prev0_l)
        out[f"h{idx}_pre_actions"] = np.stack(acts_pre)
        out[f"h{idx}_prev"] = np.stack(prev_l)
        out[f"h{idx}_power"] = np.stack(power_l)
        out[f"h{idx}_actions"] = acts
        out[f"h{idx}_values"] = vals
    out["n_cases"] = np.array(len(specs))
    np.savez_compressed(os.path.join(OUT, "haal_variants.npz"), **out)


def gen_replay_buffer():
    """ReplayBuffer (components/episode_buffer.py:237-277): ring inserts of EpisodeBatches
    of 2, 2 and 3 episodes into a 5-episode buffer (the last one wraps: split insert), the
    buffer's contents and counters after each insert, then sample(3) under
    np.random.seed(7) and sample(5) (= the whole buffer)."""
    import torch as th
    from components.episode_buffer import EpisodeBatch, ReplayBuffer
    from components.transforms import OneHot
    n, m, T = 3, 5, 4
    scheme = {"obs": {"vshape": 7, "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
              "avail_actions": {"vshape": (m,), "group": "agents", "dtype": th.int},
              "rewards": {"vshape": (n,)},
              "terminated": {"vshape": (1,), "dtype": th.uint8},
              "beta": {"vshape": (n, m)}}
    groups = {"agents": n}
    pre = {"actions": ("actions_onehot", [OneHot(out_dim=m)])}
    rng = np.random.RandomState(5)
    buf = ReplayBuffer(scheme, groups, 5, T + 1, preprocess=pre, device="cpu")
    out = {}
    for k, bs in enumerate([2, 2, 3]):
        eb = EpisodeBatch(scheme, groups, bs, T + 1, preprocess=pre, device="cpu")
        inp = {}
        for t in range(T + 1):
            d = {"obs": rng.standard_normal((bs, n, 7)).astype(np.float32),
                 "avail_actions": rng.randint(0, 2, size=(bs, n, m)).astype(np.int32),
                 "beta": rng.uniform(size=(bs, n, m)).astype(np.float32)}
            if t < T:
                d.update(actions=rng.randint(0, m, size=(bs, n, 1)).astype(np.int64),
                         rewards=rng.standard_normal((bs, n)).astype(np.float32),
                         terminated=np.full((bs, 1), t == T - 1, dtype=np.uint8))
            eb.update({kk: th.from_numpy(v) for kk, v in d.items()}, ts=t)
            for kk, v in d.items():
                inp.setdefault(kk, []).append(v)
        for kk, v in inp.items():
            out[f"ins{k}__{kk}"] = np.stack(v, axis=1)
        buf.insert_episode_batch(eb)
        for kk, v in buf.data.transition_data.items():
            out[f"after{k}__{kk}"] = v.numpy().copy()  # the buffer is overwritten in place later
        out[f"after{k}__counters"] = np.array([buf.buffer_index, buf.episodes_in_buffer])
    np.random.seed(7)
    s = buf.sample(3)
    for kk, v in s.data.transition_data.items():
        out[f"sample3__{kk}"] = v.numpy().copy()
    s = buf.sample(5)
    for kk, v in s.data.transition_data.items():
        out[f"sample5__{kk}"] = v.numpy().copy()
    out["cfg"] = np.array([n, m, T, 5])
    np.savez_compressed(os.path.join(OUT, "replay_buffer.npz"), **out)


if __name__ == "__main__":
    _install_stubs()
    if sys.argv[1:] == ["real_env"]:  # regenerate only the RealConstellationEnv fixtures
        gen_real_env()
        gen_real_variants()
        gen_real_runner_dumps()
        sys.exit(0)
    if sys.argv[1:] == ["round6"]:  # bids_as_actions on the real-env family (round 6)
        gen_real_bids()
        gen_haal_variants()
        sys.exit(0)
    if sys.argv[1:] == ["yaml"]:  # the reference's unchanged mock algorithm configs (round 4)
        gen_yaml_runner_dumps()
        sys.exit(0)
    if sys.argv[1:] == ["round2"]:  # the selector / buffer fixtures added in round 2
        gen_filtered_selectors()
        gen_haal()
        gen_replay_buffer()
        sys.exit(0)
    gen_real_env()
    gen_real_variants()
    gen_real_bids()
    gen_mt_words()
    gen_mock_reset()
    gen_mock_step()
    gen_lsa()
    gen_runner_dumps()
    gen_real_runner_dumps()
    gen_filtered_selectors()
    gen_haal()
    gen_haal_variants()
    gen_replay_buffer()
    gen_yaml_runner_dumps()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
