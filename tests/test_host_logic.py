"""Host-side mirror of the reference interfaces (CPU): EpisodeBatch layout/semantics
against the reference's own batch dumps, time-major storage equivalence, ReplayBuffer,
schedules, OneHot, scheme -- and the CPU-baseline port against the golden vectors."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from marl_sap_amd.components import DecayThenFlatSchedule, EpisodeBatch, OneHot, ReplayBuffer
from marl_sap_amd.envs.assign_env import make_scheme


def _batch(n, m, T, L=3, B=2, time_major=False, bids=False):
    scheme, pre = make_scheme(n, m, L, bids)
    return EpisodeBatch(scheme, {"agents": n}, B, T + 1, preprocess=pre, device="cpu", time_major=time_major)


def test_layout_matches_reference_dump(golden):
    g = golden("runner_dumps")
    for tag in ["ep_eg_4", "par_sap_8"]:
        n, m, T, B = [int(x) for x in g[f"{tag}__cfg"][:4]]
        b = _batch(n, m, T, B=B)
        for k, v in b.data.transition_data.items():
            ref = g[f"{tag}__{k}"]
            assert tuple(v.shape) == ref.shape, k
            assert str(v.dtype).replace("torch.", "") == str(ref.dtype), k


def test_bench_store_ceiling_and_sap_steps(monkeypatch, tmp_path):
    """The fused roofline's store_ceiling block (writes = all bytes but h in and the actions row
    the kernel keeps in LDS, against the newest tools/store_bw.hip record) and the SAP step
    counts' fast / exact split (low / high 16 bits of asg_sap_select's path_steps_out)."""
    import json
    import types
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r4_store_bw_s1.txt").write_text("# x\n" + json.dumps({"GBps": 4000.0}) + "\n")
    (prof / "r4_store_bw_s2.txt").write_text(json.dumps({"GBps": 4500.0}) + "\n" + json.dumps({"GBps": 5000.0}) + "\n")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.store_ceiling() == (5000.0, "r4_store_bw_s2.txt")
    a = types.SimpleNamespace(n=64, m=64, L=3)
    E = 16384
    roof = bench.fused_roofline(a, E, 0.5)
    per = (bench.step_bytes(64, 64, 3) + 64 * (2 * 4 * 64 + 8)) * E
    writes = per - 64 * 4 * 64 * E - 8 * 64 * E
    sc = roof["store_ceiling"]
    assert roof["bytes_per_launch"] == per and sc["write_bytes_per_launch"] == writes
    assert sc["frac"] == pytest.approx(writes / 0.5e-3 / 1e9 / 5000.0, rel=1e-3)
    # SAP step-count split as bench.run_leg decodes it
    import torch
    cs = torch.tensor([(3 << 16) | 700, 650, (1200 << 16) | 900], dtype=torch.int32).long()
    assert int((cs & 0xFFFF).sum()) == 2250 and int((cs >> 16).sum()) == 1203 and int(((cs >> 16) > 0).sum()) == 2
    res = {"path_steps_per_launch": 3453, "path_steps_fast": 2250, "path_steps_exact": 1203, "exact_problems": 2,
           "lsa_ms": 0.5}
    monkeypatch.setattr(bench, "pmc_lookup", lambda pattern, **kw: None)
    r = bench.lsa_roofline(a, 3, res)
    assert r["path_steps_fast"] == 2250 and r["path_steps_exact"] == 1203 and r["problems_on_exact_solver"] == 2


@pytest.mark.parametrize("time_major", [False, True])
def test_update_and_slicing_semantics(time_major):
    n, m, T = 3, 4, 5
    b = _batch(n, m, T, B=3, time_major=time_major)
    obs = np.arange(3 * n * 4 * m, dtype=np.float64).reshape(3, n, 4 * m)
    b.update({"obs": list(obs), "beta": [np.ones((n, m))] * 3}, ts=2)
    assert (b["filled"][:, 2] == 1).all() and b["filled"].sum() == 3
    np.testing.assert_array_equal(b["obs"][:, 2].numpy(), obs.astype(np.float32))
    b.update({"actions": torch.tensor([[0, 1, 3]] * 3)}, ts=2, mark_filled=False)
    assert b["actions_onehot"].dtype == torch.int64
    assert b["actions_onehot"][0, 2].tolist() == [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1]]
    b.update({"actions": torch.tensor([[2, 2, 2]])}, bs=[1], ts=3, mark_filled=False)
    assert b["actions"][1, 3, :, 0].tolist() == [2, 2, 2] and b["actions"][0, 3].sum() == 0
    sub = b[1:3, 2:4]
    assert sub.batch_size == 2 and sub.max_seq_length == 2 and sub["obs"].shape == (2, 2, n, 4 * m)
    with pytest.raises(ValueError):
        b.update({"obs": [np.zeros((n + 1, 4 * m))] * 3}, ts=0)
    with pytest.raises(KeyError):
        b.update({"nope": [0]}, ts=0)
    if time_major:  # one time step of all envs is one contiguous slab
        assert b["obs"][:, 2].is_contiguous()


def test_replay_buffer_ring():
    n, m, T = 2, 3, 2
    scheme, pre = make_scheme(n, m, 1)
    rb = ReplayBuffer(scheme, {"agents": n}, 5, T + 1, preprocess=pre)
    for ep in range(4):
        b = EpisodeBatch(scheme, {"agents": n}, 2, T + 1, preprocess=pre, time_major=True)
        b.update({"actions": torch.full((2, n), ep % m)}, ts=0)
        rb.insert_episode_batch(b)
    assert rb.episodes_in_buffer == 5 and rb.buffer_index == 3
    assert rb.can_sample(5) and not rb.can_sample(6)
    assert rb["actions"][:, 0, 0, 0].tolist() == [2, 3 % m, 3 % m, 1, 2]
    s = rb.sample(3, rng=np.random.RandomState(0))
    assert s.batch_size == 3


def test_schedule_onehot_scheme():
    s = DecayThenFlatSchedule(1.0, 0.05, 100, decay="linear")
    assert s.eval(0) == 1.0 and abs(s.eval(50) - 0.525) < 1e-12 and s.eval(1000) == 0.05
    oh = OneHot(5)
    assert oh.infer_output_info((1,), torch.int64) == ((5,), torch.int64)
    assert oh.transform(torch.tensor([[3], [0]])).tolist() == [[0, 0, 0, 1, 0], [1, 0, 0, 0, 0]]
    scheme, pre = make_scheme(4, 6, 3, bids_as_actions=True)
    assert scheme["actions"]["vshape"] == (6,) and pre == {}
    scheme, pre = make_scheme(4, 6, 3)
    assert scheme["obs"]["vshape"] == 24 and scheme["beta"]["part_of_state"]


def test_cpu_baseline_port_matches_golden(golden):
    """The timed CPU baseline (oracle/cpu_parallel_runner.py) is the reference algorithm."""
    from oracle.cpu_parallel_runner import NumpyMockEnv
    g = golden("mock_reset")
    for c in (0, 5, 9):
        n, m, T, L, s = [int(x) for x in g[f"c{c}_shape"]]
        np.random.seed(s)
        env = NumpyMockEnv(n, m, T, L, 0.5)
        env.reset()
        np.testing.assert_array_equal(env.sat_prox_mat, g[f"c{c}_table"])
        np.testing.assert_array_equal(env.prev_assigns, g[f"c{c}_prev_assigns"])
    st = golden("mock_step")
    c = 2
    n, m, T, L = [int(x) for x in st[f"c{c}_spec"]]
    env = NumpyMockEnv(n, m, T, L, float(st[f"c{c}_lambda"]))
    env.sat_prox_mat = st[f"c{c}_table"]
    env.k, env.curr_assignment = 0, np.zeros((n, m))
    env.beta, env.prev_assigns = env.sat_prox_mat[:, :, 0], st[f"c{c}_prev0"]
    for t in range(T):
        r, d, _ = env.step(list(st[f"c{c}_actions"][t]))
        np.testing.assert_array_equal(np.array(r), st[f"c{c}_rewards"][t])


def test_cpu_baseline_runs():
    from oracle.cpu_parallel_runner import run_parallel_baseline
    rate, steps, secs, reset_secs = run_parallel_baseline(n=4, m=4, T=3, L=1, workers=2, episodes=1)
    assert steps == 6 and rate > 0


def test_real_env_schemes_match_reference_sizes(golden):
    """RealConstellationEnv-family schemes (real_constellation_env.py:74-97,
    real_power_constellation_env.py:95-116): float16 obs of get_obs_size(), int16
    actions / prev_assigns, [n, m, L] beta, power_states only for the power variants."""
    import torch
    from marl_sap_amd.envs.real_env import make_real_scheme, obs_size
    d = golden("real_env")
    for c in range(int(d["n_cases"])):
        n, m, T, L, N, M = (int(x) for x in d[f"r{c}_spec"])
        scheme, pre = make_real_scheme(n, m, L, N, M)
        assert scheme["obs"]["vshape"] == obs_size(N, M, L) == int(d[f"r{c}_obs_size"]) == d[f"r{c}_obs0"].shape[1]
        assert scheme["obs"]["dtype"] == torch.float16 and scheme["actions"]["dtype"] == torch.int16
        assert scheme["beta"]["vshape"] == (n, m, L) and "power_states" not in scheme
        assert pre["actions"][0] == "actions_onehot"
    v = golden("real_variants")
    for c in range(int(v["n_cases"])):
        n, m, T, L, N, M = (int(x) for x in v[f"v{c}_spec"])
        scheme, _ = make_real_scheme(n, m, L, N, M, power=True)
        assert scheme["obs"]["vshape"] == int(v[f"v{c}_obs_size"]) == v[f"v{c}_obs0"].shape[1]
        assert scheme["power_states"]["vshape"] == (n,) and scheme["power_states"]["dtype"] == torch.float16


def test_bench_accounting():
    """The algorithmic figures bench.py divides by."""
    import bench
    assert bench.step_bytes(64, 64, 3) == 120073
    assert bench.step_bytes(16, 16, 3) == 16 * 16 * 29 + 16 * 20 + 9
    assert bench.agent_flops(64, 64, 3, onehot=False) == 90112  # 2 * (256*64 + 2*3*64*64 + 64*64)
    assert bench.agent_flops(64, 64, 3) == 81920  # the one-hot block is a W1 column gather
    # roof: f32 MFMA everywhere, or the GRU's 49,152 flops at 2.5 PF / 6 (split bf16)
    assert bench.agent_peak(64, 64, 3, 0) == pytest.approx(157.3)
    assert bench.agent_peak(64, 64, 3, 1) == pytest.approx(81920 / (32768 / 157.3 + 49152 / (2500 / 6)))


def test_bench_profile_order_and_reset_share(monkeypatch):
    """pmc_lookup takes the newest summary by (round, session) -- s10 after s9 -- and the
    fused roofline's PMC traffic carries the same reset share as its bytes_per_launch."""
    import types
    import bench
    names = ["pmc_step_kernel.json", "r3_pmc_x_s9.json", "r3_pmc_x_s10.json", "r2_pmc_x_s4.json",
             "r3_pmc_x_256_s2.json", "r4_pmc_x_s1.json"]
    order = sorted(names, key=bench.profile_order)
    assert order == ["pmc_step_kernel.json", "r2_pmc_x_s4.json", "r3_pmc_x_256_s2.json", "r3_pmc_x_s9.json",
                     "r3_pmc_x_s10.json", "r4_pmc_x_s1.json"]
    a = types.SimpleNamespace(n=256, m=256, L=3)
    E, spl = 2048, 20
    step = bench.step_bytes(256, 256, 3) + 256 * (2 * 4 * 64 + 8)
    rb = bench.reset_bytes(256, 256, 3)
    # a profiled launch = reset + 20 steps, measured at 1.02x its algorithmic bytes
    prof = {"hbm_bytes_per_launch": 1.02 * E * (spl * step + rb), "steps_per_launch": spl, "_path": "r4_x_s1.json"}
    monkeypatch.setattr(bench, "pmc_lookup", lambda pattern, **kw: prof if "rollout_kernel" in pattern else None)
    for rps in (0.0, 1.0 / spl):
        roof = bench.fused_roofline(a, E, 1.0, resets_per_step=rps)
        # the profile's reset share swapped for the window's: the ratio stays near 1.02
        assert roof["traffic_over_algorithmic"] == pytest.approx(1.02, abs=0.002)
        assert roof["traffic"] / roof["bytes_per_launch"] == pytest.approx(1.02, abs=0.002)


def test_bench_bids_and_q_accounting(monkeypatch):
    """The step_q rooflines: the Q rows are reported beside the HBM bytes (q_buffer), and the
    bids_as_actions env's step writes no int64 one-hot and reads the int32 assignments instead of
    the int64 actions row; no PMC summary is matched for it."""
    import types
    import bench
    monkeypatch.setattr(bench, "pmc_lookup", lambda pattern, **kw: None)
    a = types.SimpleNamespace(n=64, m=64, L=3)
    E = 16384
    q = bench.fused_roofline(a, E, 0.5, use_rnn=False, q_out=True)
    b = bench.fused_roofline(a, E, 0.5, use_rnn=False, q_out=True, bids=True)
    base = bench.step_bytes(64, 64, 3) + 64 * (4 * 64 + 8)
    assert q["bytes_per_launch"] == base * E
    assert b["bytes_per_launch"] == (base - 8 * 64 * 64 - 4 * 64) * E
    assert q["q_buffer"]["bytes_per_launch"] == 4 * 64 * 64 * E == b["q_buffer"]["bytes_per_launch"]
    assert q["traffic"] is None and b["traffic"] is None
    for r in (q, b):
        assert 0 < r["frac"] <= 1 and r["store_ceiling"]["frac"] <= 1


@pytest.mark.parametrize("time_major", [False, True])
def test_replay_buffer_matches_reference(golden, time_major):
    """Ring inserts (a split insert included), counters and seeded sample() against the
    reference ReplayBuffer's own outputs (tests/golden/replay_buffer.npz)."""
    from tests.replay_fixture import check_against_reference
    check_against_reference(golden("replay_buffer"), "cpu", time_major)


def test_continuous_selector_cpu():
    from types import SimpleNamespace
    import torch
    from marl_sap_amd.action_selectors import REGISTRY
    args = SimpleNamespace(epsilon_start=0.5, epsilon_finish=0.1, epsilon_anneal_time=100, evaluation_epsilon=0.0)
    sel = REGISTRY["continuous"](args)
    x = torch.randn(4, 3, 5)
    assert torch.equal(sel.select_action(x, None, 0, test_mode=True), x)
    torch.manual_seed(0)
    y = sel.select_action(x, None, 200)  # annealed to epsilon_finish
    assert sel.variance == 0.1 and 0.05 < float((y - x).std()) < 0.15


@pytest.mark.parametrize("selector", ["epsilon_greedy_sap_test", "sap"])
def test_jumpstart_flips_keep_reference_stream_order(selector):
    """JumpstartMAC pre-draws an episode's coin flips only when its RL MAC fuses (the
    epsilon-greedy selector and the fused SAP selector draw nothing from numpy's global
    stream).  With an RL selector that does draw (EpsilonGreedySAPTestActionSelector,
    reference sap_selectors.py:36) nothing is pre-drawn: each step draws its flip, then the
    selector its own -- the reference's order (jumpstart_controller.py:33)."""
    from types import SimpleNamespace
    import numpy as np
    import torch
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    n, m, T = 4, 4, 5
    args = SimpleNamespace(n=n, m=m, T=T, agent="rnn", hidden_dim=64, use_rnn=True, obs_last_action=False,
                           obs_agent_id=False, agent_output_type="q", action_selector=selector, seed=0,
                           epsilon_start=0.5, epsilon_finish=0.5, epsilon_anneal_time=1, evaluation_epsilon=0.0,
                           jumpstart_action_selector="haa_selector", jumpstart_epsilon_start=0.5,
                           jumpstart_epsilon_finish=0.5, jumpstart_epsilon_anneal_time=1,
                           jumpstart_evaluation_epsilon=0.0, fused_rollout=True)
    scheme = {"obs": {"vshape": m * 4}, "actions_onehot": {"vshape": (m,)}}
    mac = mac_REGISTRY["jumpstart_mac"](scheme, {"agents": n}, args)
    env = SimpleNamespace(T=T, m=m, can_step_select=lambda **k: True)
    batch = SimpleNamespace(time_major=True)
    np.random.seed(123)
    with torch.no_grad():
        mode = mac.fused_mode(env, batch, 0)
    if selector == "sap":
        # the step_q schedule (asg_step_forward + the SAP kernel): the T flips are the stream's
        # first T draws, consumed in step order
        assert mode == "step_q"
        np.random.seed(123)
        assert mac._flips == list(np.random.rand(T) < 0.5)
        return
    assert mode is None and mac._flips == []
    # nothing drawn yet: the next draw is the stream's first
    first = np.random.rand()
    np.random.seed(123)
    assert np.random.rand() == first
    # per step: the flip is drawn when the step runs
    np.random.seed(7)
    flips = [mac._coin(0, False) for _ in range(3)]
    np.random.seed(7)
    assert flips == list(np.random.rand(3) < 0.5)


def test_runner_flush_clears_env_error_when_selector_raises():
    """when a selector's status raises in flush_pending, the env's sticky device error
    is still read and cleared (chained as the cause) and the pending episodes are dropped, so the
    next flush sees neither a stale error nor duplicate episodes."""
    from marl_sap_amd.runners.gpu_runner import GpuVecRunner

    class Sel:
        def __init__(self):
            self.fail = True

        def flush(self):
            if self.fail:
                self.fail = False
                raise ValueError("matrix contains invalid numeric entries")

    class Env:
        def __init__(self):
            self.err, self.syncs = True, 0

        def sync(self):
            self.syncs += 1
            if self.err:
                self.err = False
                raise ValueError("an action outside [0, m) was passed to step")

    r = object.__new__(GpuVecRunner)
    r.mac = SimpleNamespace(action_selector=Sel())
    r.env = Env()
    r._pending, r._pending_steps = [("returns", False)], [20]
    with pytest.raises(ValueError, match="invalid numeric entries") as ei:
        r.flush_pending()
    assert isinstance(ei.value.__cause__, ValueError) and "outside" in str(ei.value.__cause__)
    assert r.env.syncs == 1 and not r.env.err
    assert r._pending == [] and r._pending_steps == []
    r.flush_pending()  # nothing stale left: no error, nothing logged twice
    assert r.env.syncs == 2


def test_sap_selector_episode_start_warm_or_cold():
    """The SAP selector's warm start carries duals from one selection to the next; the MAC's
    episode_start() (t_ep = 0) makes the next call cold when args.sap_warm_across_episodes is
    False (by default the previous episode's duals stay the start)."""
    from marl_sap_amd.action_selectors.sap_selectors import SequentialAssignmentProblemSelector
    base = dict(epsilon_start=0.1, epsilon_finish=0.1, epsilon_anneal_time=1, evaluation_epsilon=0.0)
    keep = SequentialAssignmentProblemSelector(SimpleNamespace(**base))
    keep.episode_start()
    assert not keep._cold_next
    cold = SequentialAssignmentProblemSelector(SimpleNamespace(**base, sap_warm_across_episodes=False))
    assert not cold._cold_next
    cold.episode_start()
    assert cold._cold_next
