"""The numpy Philox restatement used by the GPU action checks (oracle/philox.py) against
the published Philox4x32-10 known-answer vectors (Random123 kat_vectors), so a wrong
checker cannot agree with a wrong kernel."""
import numpy as np

from oracle.philox import eps_greedy_draws, philox4x32_10

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = philox4x32_10(*ctr, *key)
        assert tuple(int(v) for v in got) == want


def test_philox_vectorised_matches_scalar():
    rows = np.arange(1000, dtype=np.uint64) * np.uint64(7919) + np.uint64(2 ** 33)
    x, y, z, w = philox4x32_10(rows & np.uint64(0xFFFFFFFF), rows >> np.uint64(32), 6, 17, 0x1234, 0x5678)
    for i in (0, 1, 500, 999):
        r = int(rows[i])
        s = philox4x32_10(r & 0xFFFFFFFF, r >> 32, 6, 17, 0x1234, 0x5678)
        assert (int(x[i]), int(y[i]), int(z[i]), int(w[i])) == tuple(int(v) for v in s)


def test_eps_greedy_draw_rates():
    rows = np.arange(200000)
    explore, target = eps_greedy_draws(12345, rows, 3, 0.05, 64)
    assert abs(explore.mean() - 0.05) < 0.003
    assert target.min() >= 0 and target.max() < 64
    assert abs(np.bincount(target, minlength=64).std() / (len(rows) / 64)) < 0.05
    assert not eps_greedy_draws(12345, rows, 3, 0.0, 64)[0].any()
