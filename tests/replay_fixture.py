"""Replays tests/golden/replay_buffer.npz (the reference ReplayBuffer's ring inserts and
samples, tests/golden/make_golden.py:gen_replay_buffer) on this package's ReplayBuffer."""
import numpy as np
import torch

from marl_sap_amd.components import EpisodeBatch, ReplayBuffer
from marl_sap_amd.components.transforms import OneHot


def scheme_of(n, m):
    return {"obs": {"vshape": 7, "group": "agents"},
            "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
            "avail_actions": {"vshape": (m,), "group": "agents", "dtype": torch.int},
            "rewards": {"vshape": (n,)},
            "terminated": {"vshape": (1,), "dtype": torch.uint8},
            "beta": {"vshape": (n, m)}}


def check_against_reference(g, device, time_major):
    n, m, T, size = [int(x) for x in g["cfg"]]
    scheme, groups = scheme_of(n, m), {"agents": n}
    pre = {"actions": ("actions_onehot", [OneHot(out_dim=m)])}
    buf = ReplayBuffer(scheme, groups, size, T + 1, preprocess=pre, device=device)
    for k, bs in enumerate([2, 2, 3]):
        eb = EpisodeBatch(scheme, groups, bs, T + 1, preprocess=pre, device=device, time_major=time_major)
        for t in range(T + 1):
            d = {f: torch.from_numpy(g[f"ins{k}__{f}"][:, t]) for f in ("obs", "avail_actions", "beta")}
            if t < T:
                d.update({f: torch.from_numpy(g[f"ins{k}__{f}"][:, t]) for f in ("actions", "rewards", "terminated")})
            eb.update(d, ts=t)
        buf.insert_episode_batch(eb)
        np.testing.assert_array_equal([buf.buffer_index, buf.episodes_in_buffer], g[f"after{k}__counters"])
        for f, v in buf.data.transition_data.items():
            np.testing.assert_array_equal(v.cpu().numpy(), g[f"after{k}__{f}"], err_msg=f"insert {k}: {f}")
    np.random.seed(7)  # the reference samples from numpy's global stream
    for tag, bs in (("sample3", 3), ("sample5", 5)):
        s = buf.sample(bs)
        for f in s.data.transition_data:
            got = s[f]
            assert got.device.type == torch.device(device).type
            np.testing.assert_array_equal(got.cpu().numpy(), g[f"{tag}__{f}"], err_msg=f"{tag}: {f}")
