"""device-resident ReplayBuffer fed by the GPU runner's time-major
EpisodeBatch (reference: components/episode_buffer.py:237-271).  The device buffer must
hold exactly what the reference's CPU buffer holds after the same inserts (ring wrap
included) and sample the same episodes for the same numpy stream."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.components import EpisodeBatch, ReplayBuffer  # noqa: E402
from marl_sap_amd.envs import AssignEnvBatch  # noqa: E402

DEV = torch.device("cuda", 0)


def rollout(env, E, T, n):
    ep = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV, time_major=True)
    env.reset(ep, 0)
    for t in range(T):
        env.random_actions(ep, t)
        env.step(ep, t)
    env.sync()
    return ep


def test_device_replay_buffer_matches_cpu_buffer():
    n, m, T, L, E, size = 6, 8, 5, 3, 7, 16
    env = AssignEnvBatch(n, m, T, L, 0.5, num_envs=E, seed=3, device=DEV)
    gbuf = ReplayBuffer(env.scheme, {"agents": n}, size, T + 1, preprocess=env.preprocess, device=DEV)
    cbuf = ReplayBuffer(env.scheme, {"agents": n}, size, T + 1, preprocess=env.preprocess, device="cpu")
    for _ in range(4):  # 28 episodes into 16 slots: wraps twice
        ep = rollout(env, E, T, n)
        gbuf.insert_episode_batch(ep)
        cpu_ep = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device="cpu")
        for k, v in ep.data.transition_data.items():
            cpu_ep.data.transition_data[k].copy_(v.cpu())
        cbuf.insert_episode_batch(cpu_ep)
    assert (gbuf.buffer_index, gbuf.episodes_in_buffer) == (cbuf.buffer_index, cbuf.episodes_in_buffer) == (12, 16)
    for k in cbuf.data.transition_data:
        assert torch.equal(gbuf.data.transition_data[k].cpu(), cbuf.data.transition_data[k]), k
    gs = gbuf.sample(5, rng=np.random.RandomState(7))
    cs = cbuf.sample(5, rng=np.random.RandomState(7))
    for k in cs.data.transition_data:
        assert gs[k].is_cuda and torch.equal(gs[k].cpu(), cs[k]), k


@pytest.mark.parametrize("time_major", [False, True])
def test_device_replay_buffer_matches_reference(golden, time_major):
    """The device buffer against the reference ReplayBuffer's own dump: contents and
    counters after ring inserts (a split insert included), and sample() under
    np.random.seed(7) (tests/golden/replay_buffer.npz)."""
    from tests.replay_fixture import check_against_reference
    check_against_reference(golden("replay_buffer"), "cuda", time_major)
